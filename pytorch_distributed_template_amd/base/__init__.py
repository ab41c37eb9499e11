from .base_model import BaseModel  # noqa: F401
from .base_data_loader import BaseDataLoader  # noqa: F401
from .base_trainer import BaseTrainer  # noqa: F401

from .logger import setup_logging  # noqa: F401
from .visualization import TensorboardWriter  # noqa: F401

from .ddp import wrap_ddp, bucket_plan, pretune_for_ddp, is_data_parallel  # noqa: F401
from .reducer import BucketedDDP, grad_slot  # noqa: F401

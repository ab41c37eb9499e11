from .ddp import wrap_ddp, bucket_plan  # noqa: F401

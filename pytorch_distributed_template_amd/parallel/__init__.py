from .ddp import wrap_ddp, bucket_plan, pretune_for_ddp  # noqa: F401

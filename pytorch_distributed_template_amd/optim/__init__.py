"""Optimizers. ``optimizer.type`` in config resolves here first, then in torch.optim."""
from .fused import FusedSGD, FusedAdam, FusedAdamW  # noqa: F401

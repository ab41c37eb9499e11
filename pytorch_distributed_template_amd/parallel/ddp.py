"""Data parallelism over RCCL/xGMI.

Reference: ``/root/reference/train.py:45-52`` wraps the model in
``DistributedDataParallel(device_ids=[local_rank], output_device=local_rank)``
with the defaults (25 MiB buckets, ``broadcast_buffers=True``).

``wrap_ddp`` picks one of two reducers:

* ``impl="native"`` (the default on the native kernel backend): the framework's own
  reducer, ``parallel/reducer.py`` -- the native weight-gradient kernels write straight
  into 64-B-aligned bucket slots (no per-parameter copy kernels), ``ReduceOp.AVG``
  all-reduces launched from post-accumulate-grad hooks on RCCL's stream while backward
  continues, a small first bucket and a split last bucket (``docs/DDP_XGMI.md``);
* ``impl="torch"`` (the default on the stock ``torch`` backend, i.e. the reference's
  stack, and whenever a compression comm hook is asked for): torch's
  ``DistributedDataParallel`` with ``gradient_as_bucket_view`` and the same bucket size.

Either way the knobs are set for the MI355X node rather than NVSwitch defaults:

* ``bucket_cap_mb``: xGMI is a full mesh of 7 point-to-point links per GPU; RCCL's
  ring/tree channels are per-link bound, so a handful of large buckets keeps every
  channel streaming. Default 64 MiB for fp32 grads.
* ``broadcast_buffers``: the reference broadcasts BN running stats from rank 0 every
  forward (its own comment says to remove it). Configurable; the benchmark disables it
  (running stats are not used by training-mode BN).
* ``comm_hook="bf16"``: optional bf16-compressed all-reduce (half the xGMI bytes; torch
  DDP only).
* ``PDT_DDP=native|torch`` overrides the choice (A/B runs).
"""
from __future__ import annotations

import os

import torch
from torch.nn.parallel import DistributedDataParallel

from ..utils.dist import get_world_size, is_dist_ready

DEFAULT_BUCKET_MB = 64
# the first bucket (the classifier and the last stage: the gradients backward produces first)
# starts moving while the rest of backward runs
DEFAULT_FIRST_BUCKET_MB = 8


def wrap_ddp(model: torch.nn.Module, device: torch.device, bucket_cap_mb: float = DEFAULT_BUCKET_MB,
             broadcast_buffers: bool = True, gradient_as_bucket_view: bool = True,
             comm_hook: str | None = None, static_graph: bool = False,
             find_unused_parameters: bool = False, impl: str | None = None,
             first_bucket_mb: float = DEFAULT_FIRST_BUCKET_MB):
    """Wrap for data parallelism whenever a process group exists -- a 1-rank RCCL group too
    (``torchrun --nproc-per-node 1``, ``bench.py --gpus 1``): the reducer, its buckets and the
    RCCL all-reduce then run at N = 1 exactly as at N > 1. Without a process group the model
    is returned unchanged.

    ``impl``: ``"native"`` is the framework's reducer (``parallel/reducer.py``: gradients
    written by the native kernels straight into aligned bucket slots, ``ReduceOp.AVG``
    all-reduce, a small first bucket); ``"torch"`` is torch's ``DistributedDataParallel``
    with the same bucket size -- the reference's wrapper, used by default on the stock
    ``torch`` kernel backend (the reference-equivalent baseline) and for the compression
    comm hooks, which only it implements. ``None``: ``PDT_DDP`` if set, else by backend."""
    if not is_dist_ready():
        return model
    if impl is None:
        from ..ops import fused
        impl = os.environ.get("PDT_DDP") or ("torch" if fused.get_backend() == "torch" else "native")
    if comm_hook in ("bf16", "fp16"):
        impl = "torch"
    if impl == "native":
        from .reducer import BucketedDDP
        return BucketedDDP(model, device, bucket_cap_mb=bucket_cap_mb, first_bucket_mb=first_bucket_mb,
                            broadcast_buffers=broadcast_buffers)
    kwargs = dict(bucket_cap_mb=bucket_cap_mb, broadcast_buffers=broadcast_buffers,
                  gradient_as_bucket_view=gradient_as_bucket_view, static_graph=static_graph,
                  find_unused_parameters=find_unused_parameters)
    if device.type == "cuda":
        kwargs.update(device_ids=[device.index], output_device=device.index)
    ddp = DistributedDataParallel(model, **kwargs)
    if comm_hook in ("bf16", "fp16"):
        from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
        hook = default_hooks.bf16_compress_hook if comm_hook == "bf16" else default_hooks.fp16_compress_hook
        ddp.register_comm_hook(state=None, hook=hook)
    return ddp


def is_data_parallel(model) -> bool:
    from .reducer import BucketedDDP
    return isinstance(model, (DistributedDataParallel, BucketedDDP))


def pretune_for_ddp(model: torch.nn.Module, step_fn) -> None:
    """Make every rank run the same kernel variants before DDP training starts.

    ``step_fn()`` runs one forward+backward of the (unwrapped) model. Rank 0
    runs it with the tile autotuner on and broadcasts the resulting table; all
    ranks then freeze it (``ops.native_ops.pretune_distributed``). The step's
    side effects are undone: gradients are dropped and BatchNorm running stats
    restored (DDP's constructor then broadcasts rank 0's parameters/buffers).
    No-op for one rank, on CPU, or without the native library."""
    if get_world_size() <= 1:
        return
    from ..ops import fused, native_ops
    if fused.get_backend() == "torch" or not native_ops.available():
        return
    saved = [b.detach().clone() for b in model.buffers()]
    try:
        native_ops.pretune_distributed(step_fn)
    finally:
        model.zero_grad(set_to_none=True)
        with torch.no_grad():
            for b, s in zip(model.buffers(), saved):
                b.copy_(s)


def bucket_plan(model: torch.nn.Module, bucket_cap_mb: float = DEFAULT_BUCKET_MB):
    """Return the bucket sizes (bytes) DDP will build, for docs/tests."""
    import torch.distributed as dist
    params = [p for p in model.parameters() if p.requires_grad]
    limit = int(bucket_cap_mb * 1024 * 1024)
    idx, _ = dist._compute_bucket_assignment_by_size(list(reversed(params)), [1024 * 1024, limit])
    sizes = []
    rev = list(reversed(params))
    for bucket in idx:
        sizes.append(sum(rev[i].numel() * rev[i].element_size() for i in bucket))
    return sizes

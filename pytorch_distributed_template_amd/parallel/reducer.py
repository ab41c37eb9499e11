"""Bucketed gradient all-reduce for one process per GPU: the framework's own data-parallel
reducer (reference: ``/root/reference/train.py:45-52`` wraps the model in torch's
``DistributedDataParallel``).

What it does, per step:

* every trainable parameter owns a fixed SLOT in a flat fp32 bucket; slots start on 64-byte
  boundaries (the fused optimizer's 16-B vector path needs aligned gradients; torch DDP's
  bucket views are packed back to back and fall back to scalar code);
* the native backward kernels write each weight gradient STRAIGHT INTO its slot
  (``grad_slot(param)``: a fresh view of the slot, so autograd's AccumulateGrad adopts it as
  ``param.grad`` without a copy). torch DDP instead copies every gradient into its bucket with a
  scaled copy (``mul_out(bucket_view, grad, 1/world)``): 161 elementwise launches per ResNet-50
  step, ~0.75 ms at batch 2048 (``profiles/resnet50_native_bs2048_step_round3_eager.txt``).
  A gradient produced by a stock op is copied into its slot once (the fallback);
* a post-accumulate-grad hook counts the bucket's ready parameters; the last one launches
  the bucket's all-reduce asynchronously on RCCL's stream (ordered after the kernels that
  produced the gradients), so communication overlaps the rest of backward. The average is the
  collective's own ``ReduceOp.AVG`` (RCCL pre-multiplies inside the reduction kernel): no
  division launch at all. gloo has no AVG: sum, then one scale per bucket;
* a callback queued on the autograd engine runs when backward finishes: buckets with a
  parameter that received no gradient get zeros in that slot and are reduced too (so an unused
  parameter never hangs the job), then the compute stream waits for every bucket. Such a
  parameter's ``.grad`` becomes its reduced slot -- the other ranks' average when they used
  it (torch DDP's ``find_unused_parameters=True`` behaviour for a locally unused parameter),
  zeros when nobody did (torch DDP leaves ``None`` there, or errors with the reference's
  ``find_unused_parameters=False``): a weight-decaying optimizer then still decays it.
* a RETAINED gradient (``zero_grad(set_to_none=False)``, ``no_sync()``) is the slot itself;
  the native kernels then write into a scratch buffer and autograd adds it into the slot
  (``grad_out``), so accumulation sums as torch's does.

Bucket sizes are chosen for MI355X's xGMI mesh, not NVSwitch: one ring all-reduce is bound
by one ~153 GB/s link per direction and RCCL spreads channels over the 7 links, so a handful
of large buckets keeps every channel streaming. The FIRST bucket is small (the gradients that
are ready first -- the classifier -- start moving while the rest of backward runs), the others
``bucket_cap_mb`` (default 64 MiB: ResNet-50's 97.5 MiB of fp32 gradients become 1 + 2
buckets, ResNet-152's 230 MiB 1 + 4), and the LAST bucket is split so that at most 4 MiB (the
stem and first stage: ready at the very end of backward) is left exposed after backward
(ResNet-50 at bs 2048: 25.1 MiB of the last bucket are ready only at the end otherwise).
``docs/DDP_XGMI.md`` has the readiness measurements.

``broadcast_buffers`` (reference default True: BN running statistics from rank 0 before every
forward) is supported and off by default (training-mode BN never reads them). Parameters and
buffers are broadcast from rank 0 once, at construction. ``no_sync()`` accumulates gradients
locally (the next backward outside it reduces the accumulated sum). The same module runs
under HIP-graph capture: the hooks, collectives and the end-of-backward wait are recorded
like any other work on the capture stream.
"""
from __future__ import annotations

import contextlib
import hashlib
from typing import List, Optional

import torch
import torch.distributed as dist

SLOT_ALIGN = 16  # fp32 elements: every slot starts on a 64-byte boundary


class _Bucket:
    __slots__ = ("index", "flat", "params", "ready", "work", "launched")

    def __init__(self, index, flat, params):
        self.index = index
        self.flat = flat
        self.params = params
        self.ready = 0
        self.work = None
        self.launched = False


def _dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)) or \
        (t.dim() == 5 and t.is_contiguous(memory_format=torch.channels_last_3d))


def grad_slot(param: torch.Tensor) -> Optional[torch.Tensor]:
    """A new view of ``param``'s gradient slot (same sizes and strides as the parameter), or
    None when the parameter is not managed by a reducer. A fresh view per call: autograd adopts
    a returned gradient as ``param.grad`` only if nothing else references it."""
    slot = getattr(param, "_pdt_grad_slot", None)
    if slot is None:
        return None
    flat, offset = slot
    return flat.as_strided(param.shape, param.stride(), offset)


def grad_out(param: torch.Tensor, *shape, memory_format=None) -> torch.Tensor:
    """Output buffer for ``param``'s gradient: its reducer slot when there is one, the requested
    layout is the parameter's AND ``param.grad`` is None; else a new fp32 tensor of ``shape``.

    The ``param.grad is None`` condition is what keeps accumulation right: a retained
    gradient (``zero_grad(set_to_none=False)``, ``no_sync()`` micro-batches) already IS the
    slot, and autograd's AccumulateGrad will add whatever the backward returns into it --
    handing out the slot there would overwrite the retained value with g and then add g to
    itself (2g). With a separate buffer AccumulateGrad computes ``slot += g`` in place."""
    s = grad_slot(param)
    if s is not None and param.grad is None and tuple(s.shape) == tuple(shape or param.shape) and \
            (memory_format is None or s.is_contiguous(memory_format=memory_format)):
        return s
    shape = shape or tuple(param.shape)
    if memory_format is not None:
        return torch.empty(shape, dtype=torch.float32, device=param.device, memory_format=memory_format)
    return torch.empty(shape, dtype=torch.float32, device=param.device)


def plan_buckets(params: List[torch.Tensor], bucket_cap_mb: float, first_bucket_mb: float,
                 last_bucket_mb: float = 0.0) -> List[List[int]]:
    """Indices of ``params`` per bucket, in reverse registration order (the order backward
    produces gradients in); the first bucket is capped at ``first_bucket_mb``. ``last_bucket_mb``
    > 0: the LAST bucket is split so that its final part -- the gradients backward produces
    last (the stem and first stage of a CNN), whose all-reduce nothing is left to hide -- holds
    at most that much; the rest of it is reduced while those are still being computed."""
    buckets, cur, cur_bytes = [], [], 0
    cap = first_bucket_mb * 2 ** 20
    for i in reversed(range(len(params))):
        nbytes = params[i].numel() * 4
        if cur and cur_bytes + nbytes > cap:
            buckets.append(cur)
            cur, cur_bytes = [], 0
            cap = bucket_cap_mb * 2 ** 20
        cur.append(i)
        cur_bytes += nbytes
    if cur:
        buckets.append(cur)
    if last_bucket_mb > 0 and len(buckets) > 1:
        last, tail_bytes, cut = buckets[-1], 0, len(buckets[-1])
        while cut > 1 and tail_bytes + params[last[cut - 1]].numel() * 4 <= last_bucket_mb * 2 ** 20:
            cut -= 1
            tail_bytes += params[last[cut]].numel() * 4
        if 0 < cut < len(last):
            buckets[-1:] = [last[:cut], last[cut:]]
    return buckets


class BucketedDDP(torch.nn.Module):
    """Data-parallel wrapper over a process group (RCCL on GPUs, gloo on CPU): same contract as
    the torch DDP wrapper the reference uses -- ``.module``, forward passthrough, gradients
    averaged over the ranks when backward returns -- with the bucketing above."""

    # every gradient ends in a fixed slot: a graph-captured step may drop the gradients
    # (``zero_grad(set_to_none=True)``) and still see the same addresses on every replay
    static_grad_slots = True

    def __init__(self, module: torch.nn.Module, device: torch.device | None = None, process_group=None,
                 bucket_cap_mb: float = 64.0, first_bucket_mb: float = 8.0, broadcast_buffers: bool = False,
                 last_bucket_mb: float = 4.0):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.world = dist.get_world_size(process_group)
        self.broadcast_buffers = broadcast_buffers
        self.device = device if device is not None else next(module.parameters()).device
        self._avg = dist.get_backend(process_group) == "nccl"  # RCCL: ReduceOp.AVG; gloo: SUM + scale
        self._sync = True
        self._in_backward = False
        self.fallback_copies = 0  # gradients that had to be copied into their slot (stock ops)
        self.fallback_shapes = set()  # their parameter shapes (bench.py records them)
        self.params = [p for p in module.parameters() if p.requires_grad]
        self._verify_shapes()
        self._broadcast_state()
        self.bucket_index = plan_buckets(self.params, bucket_cap_mb, first_bucket_mb, last_bucket_mb)
        self.buckets: List[_Bucket] = []
        self._bucket_of = {}
        for bi, idx in enumerate(self.bucket_index):
            offs, n = [], 0
            for i in idx:
                offs.append(n)
                n += -(-self.params[i].numel() // SLOT_ALIGN) * SLOT_ALIGN
            flat = torch.zeros(n, dtype=torch.float32, device=self.device)
            bparams = []
            for i, off in zip(idx, offs):
                p = self.params[i]
                if not _dense(p):
                    raise ValueError("BucketedDDP: every parameter must be dense (no overlapping strides)")
                p._pdt_grad_slot = (flat, off)
                self._bucket_of[id(p)] = bi
                bparams.append(p)
            self.buckets.append(_Bucket(bi, flat, bparams))
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    # ------------------------------------------------------------------ setup
    def _verify_shapes(self):
        """Every rank must hold the same parameter list (else the buckets would not line up):
        [count, total elements, a digest of every parameter's shape and dtype in order] --
        fixed size whatever the parameter count -- must be equal on all ranks."""
        h = hashlib.sha256()
        for p in self.params:
            h.update(repr((tuple(p.shape), str(p.dtype))).encode())
        d = h.digest()
        sig = torch.tensor([len(self.params), sum(p.numel() for p in self.params),
                            int.from_bytes(d[:7], "little"), int.from_bytes(d[7:14], "little")], dtype=torch.int64)
        dev = self.device if self.device.type == "cuda" else torch.device("cpu")
        # MAX of (sig, -sig): every rank learns the max AND the min, so a mismatch raises on
        # EVERY rank (a broadcast from rank 0 would let rank 0 continue into the parameter
        # broadcast and wait there for the ranks that raised)
        t = torch.cat([sig, -sig]).to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.process_group)
        t = t.cpu()
        if not (torch.equal(t[:4], sig) and torch.equal(-t[4:], sig)):
            raise RuntimeError("BucketedDDP: parameter shapes differ between ranks")

    @torch.no_grad()
    def _broadcast_state(self):
        tensors = [p.detach() for p in self.module.parameters()] + [b for b in self.module.buffers()]
        if self.world > 1 and tensors:
            dist._broadcast_coalesced(self.process_group or dist.group.WORLD, tensors, 250 * 2 ** 20, 0)

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kwargs):
        if self._in_backward and torch.is_grad_enabled():
            # the previous backward raised before its final callback (e.g. a caught OOM): the
            # engine drops queued callbacks then, so the bucket state is reset here, as torch
            # DDP prepares its reducer in forward
            self._in_backward = False
            for b in self.buckets:
                if b.work is not None:
                    # an all-reduce launched before the failure may still be running on RCCL's
                    # stream over b.flat: make the compute stream wait for it before the next
                    # backward's kernels write into the same slots
                    b.work.wait()
                b.ready, b.work, b.launched = 0, None, False
        if self.broadcast_buffers and self.world > 1:
            bufs = list(self.module.buffers())
            if bufs:
                dist._broadcast_coalesced(self.process_group or dist.group.WORLD, bufs, 250 * 2 ** 20, 0)
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        """Gradients accumulate locally inside; the first backward after it reduces the sum."""
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    # ------------------------------------------------------------------ backward
    def _on_grad(self, p: torch.Tensor):
        if not self._sync:
            return
        if not self._in_backward:
            self._in_backward = True
            for b in self.buckets:
                b.ready, b.work, b.launched = 0, None, False
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        slot = grad_slot(p)
        g = p.grad
        if g.data_ptr() != slot.data_ptr() or g.stride() != slot.stride():
            # a stock op's gradient: copy it into the slot once (native kernels wrote in place)
            slot.copy_(g)
            p.grad = slot
            self.fallback_copies += 1
            self.fallback_shapes.add(tuple(p.shape))
        b = self.buckets[self._bucket_of[id(p)]]
        b.ready += 1
        if b.ready == len(b.params):
            self._launch(b)

    def _launch(self, b: _Bucket):
        b.launched = True
        # (world 1 too: the same RCCL path as every rank of an N > 1 job)
        if self._avg:
            b.work = dist.all_reduce(b.flat, op=dist.ReduceOp.AVG, group=self.process_group, async_op=True)
        else:
            b.work = dist.all_reduce(b.flat, group=self.process_group, async_op=True)

    def _finalize(self):
        for b in self.buckets:
            if not b.launched:
                # parameters that got no gradient this step: their slots contribute zeros
                for p in b.params:
                    if p.grad is None:
                        s = grad_slot(p)
                        s.zero_()
                        p.grad = s
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if not self._avg:
                    b.flat.div_(self.world)
            b.work = None
        self._in_backward = False

    # ------------------------------------------------------------------ misc
    def bucket_bytes(self) -> List[int]:
        return [b.flat.numel() * 4 for b in self.buckets]

    def state_dict(self, *args, **kwargs):
        # the same keys torch DDP produces ("module." prefix): checkpoints interchange
        return super().state_dict(*args, **kwargs)

"""Multi-tensor fused SGD / Adam(W) (+AMSGrad) on MI355X.

Reference optimizer: ``torch.optim.Adam(lr=1e-3, weight_decay=0, amsgrad=True)``
(``/root/reference/config/config.json:38-45``), stepped once per batch at
``trainer/trainer.py:58``. Semantics match torch.optim exactly (tested against
it); the state_dict format is torch's (``momentum_buffer`` / ``exp_avg`` /
``exp_avg_sq`` / ``max_exp_avg_sq`` / ``step``), so checkpoints interchange
with the torch optimizers of the same name.

On GPU one HIP kernel (``csrc/optim.hip``) updates every parameter tensor:
the host builds a chunk table once per parameter set, re-uploads pointer
tables only when a tensor moved (asynchronously, from pinned memory: nothing in
``step()`` blocks the host) and each step is a single launch that also writes the
bf16 shadow copy of each parameter that the conv/GEMM kernels consume. On CPU
(gloo plumbing) the step falls back to torch's reference implementation.

``capturable=True`` (what a HIP-graph training step needs, cf. torch's capturable
Adam): the learning rate and Adam's step count live in a small device tensor per
param group that the kernels read, so a captured ``step()`` replays with the
current lr (the host rewrites it, outside the graph, in ``refresh_scalars()`` --
called by every eager ``step()`` too) and with the bias corrections of the current
step (t is incremented on the device, in the graph). ``state_dict()`` writes the
device step count back into each parameter's ``step`` so checkpoints stay torch's.
Capturable Adam keeps ONE step count per param group, so it requires every parameter of
a group to receive a gradient on every step (a captured graph assumes that anyway):
``step()`` raises if the set of parameters with gradients changes between steps --
torch's per-parameter counts would diverge from the group count there, and a checkpoint
reloaded into torch.optim would apply different bias corrections.
"""
from __future__ import annotations

import ctypes

import os

import torch
from torch.optim import Optimizer

# elements per work-list chunk (one workgroup walks one chunk; PDT_OPT_CHUNK overrides):
# 32768 -- ResNet-50 FusedSGD step 248 us vs 289 us at 65536 (profiles/optim_chunk_round2.txt)
CHUNK = int(os.environ.get("PDT_OPT_CHUNK", "32768"))


def _bump_versions(params):
    """The step kernel writes parameters through raw pointers, invisible to
    autograd's version counters: bump them so caches keyed on ``_version``
    (fp8 weight copies, saved-tensor checks) see the update."""
    from torch.autograd.graph import increment_version
    for p in params:
        increment_version(p)


def _to_device_async(host: torch.Tensor, device) -> torch.Tensor:
    """H2D copy that never blocks the host: stage through pinned memory (the
    caching host allocator keeps the pinned block alive until the copy has run)
    -- a pageable ``.to(device)`` waits for the whole queued step to drain."""
    if device.type != "cuda":
        return host.to(device)
    return host.pin_memory().to(device, non_blocking=True)


class _Plan:
    """Device-side pointer/chunk tables for one param group.

    The chunk table depends only on the parameter sizes and is built once; the
    pointer tables are re-uploaded (asynchronously) only when a tensor moved,
    e.g. after ``zero_grad(set_to_none=True)`` handed autograd fresh gradient
    buffers at new addresses."""

    def __init__(self, params, device):
        from ..ops import native_ops
        lib = native_ops._load()
        sz = lib.pdt_chunk_struct_size()
        assert sz == 24, sz
        import numpy as np
        sizes = [p.numel() for p in params]
        nch = sum((n + CHUNK - 1) // CHUNK for n in sizes)
        arr = np.zeros(nch, dtype=[("t", "<i4"), ("pad", "<i4"), ("off", "<i8"), ("len", "<i8")])
        i = 0
        for ti, n in enumerate(sizes):
            for off in range(0, n, CHUNK):
                arr[i] = (ti, 0, off, min(CHUNK, n - off))
                i += 1
        self.device = device
        self.chunks = _to_device_async(torch.from_numpy(arr.view(np.uint8).copy()), device)
        self.nchunks = nch
        self.shape_key = self._shape_key(params)
        self.tables = {}
        self.ptr_keys = {}

    @staticmethod
    def _shape_key(params):
        return tuple((id(p), p.numel()) for p in params)

    def update(self, tensors_by_role):
        for role, ts in tensors_by_role.items():
            ptrs = tuple(0 if t is None else t.data_ptr() for t in ts)
            if self.ptr_keys.get(role) != ptrs:
                self.tables[role] = _to_device_async(torch.tensor(ptrs, dtype=torch.int64), self.device)
                self.ptr_keys[role] = ptrs

    def ptr(self, role):
        t = self.tables.get(role)
        return None if t is None else t.data_ptr()


def _native_ok(params):
    from ..ops import native_ops
    return (len(params) > 0 and all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous(
        memory_format=torch.channels_last if p.dim() == 4 else torch.contiguous_format) or
        (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()) for p in params)
        and native_ops.available())


class _FusedBase(Optimizer):
    def __init__(self, params, defaults, write_bf16_shadow=True, capturable=False):
        super().__init__(params, defaults)
        self.write_bf16_shadow = write_bf16_shadow
        self.capturable = bool(capturable)
        self._plans = {}
        self._shadows = {}
        self._dev = {}      # capturable: group index -> device [lr, t]
        self._dev_lr = {}   # the lr last written into it
        self._grad_sets = {}  # capturable Adam: group index -> ids of the params stepped first

    def _dev_scalars(self, gi, group, device, t0=0.0):
        """The group's device [lr, t] (created from the host values on first use)."""
        d = self._dev.get(gi)
        if d is None:
            d = torch.tensor([float(group["lr"]), float(t0)], dtype=torch.float32, device=device)
            self._dev[gi] = d
            self._dev_lr[gi] = float(group["lr"])
        return d

    @torch.no_grad()
    def sync_shadows(self):
        """Re-form every bf16 weight shadow from its fp32 parameter and register it again.

        After parameters were written outside ``step()`` (a state restore, a checkpoint load)
        the registered shadows no longer match the parameters' versions, so the next forward
        casts each weight into a NEW buffer -- and a HIP graph captured at that point records
        those casts and repeats them on every replay (53 extra cast kernels, 0.33 ms, per
        ResNet-50 replay: ``profiles/graph_vs_eager_resnet50_round6.txt``). Called before a
        capture, the captured forward reads the shadows the captured ``step()`` rewrites."""
        if not self.write_bf16_shadow:
            return
        from ..ops import native_ops
        for group in self.param_groups:
            for p in group["params"]:
                sh = self._shadows.get(id(p))
                if sh is None or sh.data_ptr() == 0 or sh.shape != p.shape:
                    continue
                sh.copy_(p.detach())
                native_ops.register_shadow(p, sh)

    def refresh_scalars(self):
        """Write each group's current lr into its device scalars (capturable mode): call it
        before replaying a graph that captured ``step()`` -- an LR scheduler changes only the
        host value. A no-op for groups whose lr did not change (and outside capturable mode)."""
        if not self.capturable:
            return
        for gi, group in enumerate(self.param_groups):
            d = self._dev.get(gi)
            if d is not None and self._dev_lr.get(gi) != float(group["lr"]):
                d[0].fill_(float(group["lr"]))
                self._dev_lr[gi] = float(group["lr"])

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics; ``set_to_none=False`` (a graph-captured step must keep its gradient
        buffers) zeroes every gradient with one multi-tensor launch per device / dtype instead
        of one fill kernel per parameter (161 for ResNet-50)."""
        if set_to_none:
            return super().zero_grad(set_to_none=True)
        groups = {}
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    if p.grad.grad_fn is not None:
                        p.grad.detach_()
                    else:
                        p.grad.requires_grad_(False)
                    groups.setdefault((p.grad.device, p.grad.dtype), []).append(p.grad)
        for grads in groups.values():
            torch._foreach_zero_(grads)

    def _step_prologue(self):
        if self.capturable and not torch.cuda.is_current_stream_capturing():
            self.refresh_scalars()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dev.clear()  # rebuilt from the loaded lr / step on the next step()
        self._dev_lr.clear()

    def _shadow(self, p):
        if not self.write_bf16_shadow:
            return None
        s = self._shadows.get(id(p))
        if s is None or s.data_ptr() == 0:
            if p.dim() == 4:
                s = torch.empty_like(p, dtype=torch.bfloat16, memory_format=torch.channels_last)
            else:
                s = torch.empty_like(p, dtype=torch.bfloat16)
            self._shadows[id(p)] = s
        return s

    def _plan(self, gi, params, roles, device):
        plan = self._plans.get(gi)
        if plan is None or plan.shape_key != _Plan._shape_key(params):
            plan = _Plan(params, device)
            self._plans[gi] = plan
        plan.update(roles)
        return plan

    @staticmethod
    def _stream():
        return torch.cuda.current_stream().cuda_stream


class FusedSGD(_FusedBase):
    """torch.optim.SGD semantics (momentum, dampening, nesterov, weight_decay)."""

    def __init__(self, params, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 write_bf16_shadow=True, capturable=False):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(params, defaults, write_bf16_shadow, capturable)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._step_prologue()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if not _native_ok(params):
                self._torch_step(group, params)
                continue
            from ..ops import native_ops
            first = False
            bufs = []
            for p in params:
                st = self.state[p]
                if group["momentum"] != 0:
                    if "momentum_buffer" not in st or st["momentum_buffer"] is None:
                        st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                        first = True
                    bufs.append(st["momentum_buffer"])
                else:
                    bufs.append(None)
            grads = [p.grad if p.grad.dtype == torch.float32 else p.grad.float() for p in params]
            grads = [g if g.stride() == p.stride() else g.contiguous(memory_format=torch.channels_last
                                                                     if p.dim() == 4 else torch.contiguous_format)
                     for g, p in zip(grads, params)]
            shadows = [self._shadow(p) for p in params]
            roles = {"p": params, "g": grads, "b": bufs if group["momentum"] != 0 else [None] * len(params),
                     "s": shadows if self.write_bf16_shadow else [None] * len(params)}
            plan = self._plan(gi, params, roles, params[0].device)
            dev = self._dev_scalars(gi, group, params[0].device) if self.capturable else None
            rc = native_ops._load().pdt_sgd_step2(
                plan.chunks.data_ptr(), plan.nchunks, plan.ptr("p"), plan.ptr("g"),
                plan.ptr("b") if group["momentum"] != 0 else None,
                plan.ptr("s") if self.write_bf16_shadow else None,
                float(group["lr"]), float(group["momentum"]), float(group["dampening"]),
                float(group["weight_decay"]), int(group["nesterov"]), int(first), 1.0,
                dev.data_ptr() if dev is not None else None, self._stream())
            native_ops._chk(rc, "sgd_step")
            _bump_versions(params)
            if self.write_bf16_shadow:
                for p, s in zip(params, shadows):
                    native_ops.register_shadow(p, s)
        return loss

    def _torch_step(self, group, params):
        for p in params:
            g = p.grad
            if group["weight_decay"] != 0:
                g = g.add(p, alpha=group["weight_decay"])
            if group["momentum"] != 0:
                st = self.state[p]
                buf = st.get("momentum_buffer")
                if buf is None:
                    buf = torch.clone(g).detach()
                    st["momentum_buffer"] = buf
                else:
                    buf.mul_(group["momentum"]).add_(g, alpha=1 - group["dampening"])
                g = g.add(buf, alpha=group["momentum"]) if group["nesterov"] else buf
            p.add_(g, alpha=-group["lr"])


class FusedAdam(_FusedBase):
    """torch.optim.Adam semantics (L2 weight decay; ``amsgrad``)."""
    decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 write_bf16_shadow=True, capturable=False):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=amsgrad)
        super().__init__(params, defaults, write_bf16_shadow, capturable)

    def state_dict(self):
        """torch's format; in capturable mode each parameter's ``step`` is first set from the
        group's device step count (replayed graphs advance only that)."""
        if self.capturable:
            for gi, group in enumerate(self.param_groups):
                d = self._dev.get(gi)
                if d is None:
                    continue
                t = float(d[1].item())
                for p in group["params"]:
                    if p in self.state and "step" in self.state[p]:
                        self.state[p]["step"] = torch.tensor(t)
        return super().state_dict()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._step_prologue()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            b1, b2 = group["betas"]
            native = _native_ok(params)
            dev_step = self.capturable and native
            if dev_step:
                key = tuple(id(p) for p in params)
                seen = self._grad_sets.setdefault(gi, key)
                if seen != key:
                    raise RuntimeError(
                        "capturable FusedAdam: the set of parameters with gradients changed between steps "
                        f"(group {gi}: {len(seen)} -> {len(key)} params); the group's single device step "
                        "count requires every parameter to receive a gradient on every step")
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    if group["amsgrad"]:
                        st["max_exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if not dev_step:  # (capturable: the device count is the step, see state_dict)
                    st["step"] += 1
            step = float(self.state[params[0]]["step"]) if not dev_step else 1.0
            bc1 = 1 - b1 ** step
            bc2 = 1 - b2 ** step
            if not native:
                self._torch_step(group, params, bc1, bc2)
                continue
            from ..ops import native_ops
            grads = [p.grad if p.grad.dtype == torch.float32 else p.grad.float() for p in params]
            grads = [g if g.stride() == p.stride() else g.contiguous(memory_format=torch.channels_last
                                                                     if p.dim() == 4 else torch.contiguous_format)
                     for g, p in zip(grads, params)]
            shadows = [self._shadow(p) for p in params]
            roles = {"p": params, "g": grads, "m": [self.state[p]["exp_avg"] for p in params],
                     "v": [self.state[p]["exp_avg_sq"] for p in params],
                     "vm": [self.state[p].get("max_exp_avg_sq") for p in params] if group["amsgrad"]
                     else [None] * len(params),
                     "s": shadows if self.write_bf16_shadow else [None] * len(params)}
            plan = self._plan(gi, params, roles, params[0].device)
            dev = self._dev_scalars(gi, group, params[0].device, t0=float(self.state[params[0]]["step"])) \
                if dev_step else None
            rc = native_ops._load().pdt_adam_step2(
                plan.chunks.data_ptr(), plan.nchunks, plan.ptr("p"), plan.ptr("g"), plan.ptr("m"), plan.ptr("v"),
                plan.ptr("vm") if group["amsgrad"] else None, plan.ptr("s") if self.write_bf16_shadow else None,
                float(group["lr"]), float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                int(self.decoupled), float(bc1), float(bc2), 1.0, dev.data_ptr() if dev is not None else None,
                int(dev is not None), self._stream())
            native_ops._chk(rc, "adam_step")
            _bump_versions(params)
            if self.write_bf16_shadow:
                for p, s in zip(params, shadows):
                    native_ops.register_shadow(p, s)
        return loss

    def _torch_step(self, group, params, bc1, bc2):
        b1, b2 = group["betas"]
        for p in params:
            st = self.state[p]
            g = p.grad
            if group["weight_decay"] != 0:
                if self.decoupled:
                    p.mul_(1 - group["lr"] * group["weight_decay"])
                else:
                    g = g.add(p, alpha=group["weight_decay"])
            st["exp_avg"].mul_(b1).add_(g, alpha=1 - b1)
            st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
            v = st["exp_avg_sq"]
            if group["amsgrad"]:
                torch.maximum(st["max_exp_avg_sq"], v, out=st["max_exp_avg_sq"])
                v = st["max_exp_avg_sq"]
            denom = (v.sqrt() / (bc2 ** 0.5)).add_(group["eps"])
            p.addcdiv_(st["exp_avg"], denom, value=-group["lr"] / bc1)


class FusedAdamW(FusedAdam):
    """torch.optim.AdamW semantics (decoupled weight decay)."""
    decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 write_bf16_shadow=True, capturable=False):
        super().__init__(params, lr, betas, eps, weight_decay, amsgrad, write_bf16_shadow, capturable)

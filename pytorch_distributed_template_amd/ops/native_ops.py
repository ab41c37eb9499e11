"""ctypes bindings to ``libpdt_hip.so`` and the autograd Functions built on them.

Every op checks shapes / dtypes / memory formats on the host before a kernel
is launched (a mis-shaped launch on MI355X can fault the whole node) and
raises loudly if the library is missing on a GPU run -- there is no silent
fallback inside this module. ``ops/fused.py`` decides native vs torch.

Tensor conventions: activations are bf16 ``channels_last`` (NHWC storage);
parameters stay fp32 (master weights) and are cast to bf16 shadows that the
kernels read; gradients of parameters are produced in fp32.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from pathlib import Path

import torch
import torch.nn as nn

_LIB_PATH = Path(os.environ.get("PDT_LIB_PATH", "") or
                 Path(__file__).resolve().parents[1] / "_lib" / "libpdt_hip.so")  # override: A/B builds
_lib = None
_lock = threading.Lock()

c_int, c_long, c_float, c_double, c_void_p, c_uint = (ctypes.c_int, ctypes.c_long, ctypes.c_float,
                                                      ctypes.c_double, ctypes.c_void_p, ctypes.c_uint)
P = c_void_p

_SIGS = {
    "pdt_conv_nt_ax": (c_int, [P] * 4 + [c_int] * 11 + [P] * 6 + [c_int] * 3 + [c_int] + [P] * 9 + [P]),
    "pdt_conv_nt_ax2": (c_int, [P] * 4 + [c_int] * 25 + [P] * 6 + [c_int] * 3 + [c_int] + [P] * 9 + [P]),
    "pdt_conv_nt_ax3": (c_int, [P] * 6 + [c_int] * 25 + [P] * 6 + [c_int] * 3 + [c_int] + [P] * 9 + [P]),
    "pdt_stem_fwd_rows": (c_int, [c_int, c_int, c_int, c_int]),
    "pdt_stem_fwd": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P]),
    "pdt_stem_wgrad_splits": (c_int, [c_int, c_int, c_int, c_int]),
    "pdt_stem_wgrad": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, P]),
    "pdt_stem_wgrad_v": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "pdt_stem_wgrad_splits_v": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "pdt_conv_nt_stat_rows": (c_int, [c_int, c_int, c_int, c_int]),
    "pdt_conv_nt_bnb_rows": (c_int, [c_int, c_int, c_int, c_int]),
    "pdt_conv_nt_num_variants": (c_int, []),
    "pdt_conv_nt_variant_kind": (c_int, [c_int]),
    "pdt_conv_nt_resolve_variant": (c_int, [c_int, c_int, c_int, c_int]),
    "pdt_conv_nt": (c_int, [P, P, P, P, P, P, P] + [c_int] * 25 + [P, c_int, c_int, P]),
    "pdt_conv_nt_bnb": (c_int, [P] * 5 + [c_int] * 25 + [P] * 6 + [c_int] * 3 + [P]),
    "pdt_conv_nt_bnb2": (c_int, [P] * 5 + [c_int] * 25 + [P] * 6 + [c_int] * 3 + [P] * 3 + [P]),
    "pdt_conv_nt_bnb_supports": (c_int, [c_int] * 5),
    "pdt_ln_fwd": (c_int, [P, P, P, P, P, P, c_int, c_int, c_float, P]),
    "pdt_gemm_f8_q8": (c_int, [P] * 6 + [c_int] * 8 + [P, P, c_int, P, P, P, c_int, c_int, P, P]),
    "pdt_gemm_f8_q8_cs": (c_int, [P] * 6 + [c_int] * 8 + [P, P, c_int, P, P, P, c_int, c_int, P, P, P]),
    "pdt_gemm_f8_bm": (c_int, [c_int]),
    "pdt_cast_cs_bands": (c_int, [c_int]),
    "pdt_cast_fp8_delayed_cs": (c_int, [P, c_int, c_int, P, c_int, P, P, P, P, P]),
    "pdt_wgrad_reduce_rows": (c_int, [P, P, c_int, c_int, c_float, c_int, P, P]),
    "pdt_reduce_rows_work": (c_long, [c_int, c_int]),
    "pdt_gemm_f8_q8_part": (c_long, [c_int, c_int]),
    "pdt_ln_bwd_f8": (c_int, [P] * 9 + [c_int, c_int, c_int] + [P] * 6),
    "pdt_ln_bwd_f8_db": (c_int, [P] * 9 + [c_int, c_int, c_int] + [P] * 7 + [c_int, P]),
    "pdt_wgrad_f8_num_variants": (c_int, []),
    "pdt_wgrad_f8_plan": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)]),
    "pdt_wgrad_f8_workspace": (c_long, [c_int, c_int, c_int]),
    "pdt_linear_wgrad_f8": (c_int, [P] * 8 + [c_int] * 9 + [P]),
    "pdt_bn_bwd_apply_dual": (c_int, [P] * 12 + [c_long, c_int, P]),
    "pdt_bn_apply_res_affine": (c_int, [P] * 7 + [c_long, c_int, c_int, P, P]),
    "pdt_ln_fwd_f8": (c_int, [P, P, P, P, P, P, c_int, c_int, c_float, P, P, P, P, P]),
    "pdt_ln_add_fwd": (c_int, [P] * 8 + [c_int, c_int, c_float] + [P] * 5),
    "pdt_ln_fwd_f8_blocks": (c_int, [c_int]),
    "pdt_fp8_meta_roll_partial": (c_int, [P, P, c_int, c_int, P, P]),
    "pdt_ln_bwd_blocks": (c_int, [c_int]),
    "pdt_ln_bwd": (c_int, [P] * 9 + [c_int, c_int, c_int, P, P]),
    "pdt_gelu_bwd": (c_int, [P, P, P, c_long, P]),
    "pdt_wgrad_plan": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)]),
    "pdt_wgrad_plan2": (c_int, [c_int] * 7 + [ctypes.POINTER(c_int)]),
    "pdt_wgrad_num_variants": (c_int, []),
    "pdt_wgrad_halo_id": (c_int, []),
    "pdt_wgrad_ring_id": (c_int, []),
    "pdt_wgrad_workspace": (c_long, [c_int, c_int, c_int]),
    "pdt_wgrad_reduce": (c_int, [P, P, P, P, c_int, c_int, c_int, c_float, c_int, P]),
    "pdt_conv_wgrad": (c_int, [P, P, P, P] + [c_int] * 16 + [c_int, c_int, c_float, c_int, c_int, c_int, P, P]),
    "pdt_conv_wgrad2": (c_int, [P, P, P, P] + [c_int] * 16 + [c_int, c_int, c_float, c_int, c_int, c_int, P, P, P,
                                                                P]),
    "pdt_bn_stats_blocks": (c_int, [c_long, c_int]),
    "pdt_bn_bwd_reduce_pool": (c_int, [P] * 7 + [c_int] * 10 + [P]),
    "pdt_bn_bwd_apply_pool": (c_int, [P] * 9 + [c_int] * 9 + [P]),
    "pdt_rows_reduce_workspace": (c_long, [c_int, c_int]),
    "pdt_bn_stats": (c_int, [P, P, c_long, c_int, c_int, P]),
    "pdt_bn_finalize": (c_int, [P, c_int, c_int, c_double, c_float, c_float] + [P] * 9 + [P]),
    "pdt_bn_apply": (c_int, [P, P, P, P, P, c_long, c_int, c_int, P, P]),
    "pdt_bn_bwd_reduce": (c_int, [P, P, P, P, P, P, P, c_long, c_int, c_int, c_int, P, P]),
    "pdt_bn_bwd_finalize": (c_int, [P, c_int, c_int, c_double] + [P] * 8 + [c_int, P]),
    "pdt_bn_bwd_apply": (c_int, [P] * 10 + [c_long, c_int, c_int, P, P]),
    "pdt_maxpool_fwd": (c_int, [P, P, P] + [c_int] * 9 + [P]),
    "pdt_maxpool_fwd_affine": (c_int, [P] * 5 + [c_int] * 9 + [P]),
    "pdt_maxpool_bwd": (c_int, [P, P, P] + [c_int] * 9 + [P]),
    "pdt_maxpool_bwd_bnred": (c_int, [P] * 8 + [c_int] * 7 + [P]),
    "pdt_avgpool_fwd": (c_int, [P, P, c_int, c_int, c_int, P]),
    "pdt_avgpool_bwd": (c_int, [P, P, c_int, c_int, c_int, P]),
    "pdt_xent_fwd": (c_int, [P, c_int, P, P, P, P, c_int, c_int, c_float, P]),
    "pdt_xent_bwd": (c_int, [P, c_int, P, P, P, P, c_int, c_int, c_float, P]),
    "pdt_colsum": (c_int, [P, P, P, c_int, c_int, c_int, P]),
    "pdt_colsum_workspace": (c_long, [c_int, c_int]),
    "pdt_chunk_struct_size": (c_int, []),
    "pdt_sgd_step": (c_int, [P, c_int, P, P, P, P, c_float, c_float, c_float, c_float, c_int, c_int, c_float, P]),
    "pdt_adam_step": (c_int, [P, c_int, P, P, P, P, P, P] + [c_float] * 5 + [c_int, c_float, c_float, c_float, P]),
    "pdt_sgd_step2": (c_int, [P, c_int, P, P, P, P, c_float, c_float, c_float, c_float, c_int, c_int, c_float, P, P]),
    "pdt_adam_step2": (c_int, [P, c_int, P, P, P, P, P, P] + [c_float] * 5 + [c_int, c_float, c_float, c_float, P,
                                                                            c_int, P]),
    "pdt_fill_uniform_bf16": (c_int, [P, c_long, c_uint, P]),
    "pdt_cast_f32_bf16": (c_int, [P, P, c_long, P]),
    "pdt_synth_images_bf16": (c_int, [P, P, c_long, c_int, c_int, c_int, c_uint, P, c_int, P]),
    "pdt_lane_reduce_probe": (c_int, [P, P, c_int, P]),
    "pdt_wt_dgrad": (c_int, [P, P] + [c_int] * 9 + [P]),
    "pdt_transpose_cast": (c_int, [P, P, c_int, c_int, P]),
    "pdt_wt_job_size": (c_int, []),
    "pdt_wt_dgrad_multi": (c_int, [P, c_int, c_long, P]),
    "pdt_add_bf16": (c_int, [P, P, P, c_long, P]),
    "pdt_attn_fwd": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P]),
    "pdt_cls_attn_fwd": (c_int, [P, P, P, c_int, c_int, c_int, P]),
    "pdt_gemm_ring": (c_int, [P] * 6 + [c_int] * 8 + [P]),
    "pdt_cls_attn_bwd": (c_int, [P, P, P, P, P, c_int, c_int, c_int, P]),
    "pdt_attn_fwd_f8": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P]),
    "pdt_attn_fwd_tiles": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P]),
    "pdt_attn_set_bwd_single": (c_int, [c_int]),
    "pdt_gemm_f8_num_variants": (c_int, []),
    "pdt_gelu_dual_cast_fp8": (c_int, [P, c_long, P, c_int, P, P, P, P, P]),
    "pdt_cast_fp8_gelu_grad_cs": (c_int, [P, P, c_int, c_int, P, c_int, P, P, P, P, P]),
    "pdt_gemm_f8": (c_int, [P, P, P, P, P, P] + [c_int] * 8 + [P, P, c_int, P]),
    "pdt_bn_set_unroll": (c_int, [c_int]),
    "pdt_amax_blocks": (c_int, [c_long]),
    "pdt_amax_partial": (c_int, [P, c_int, c_long, P, P]),
    "pdt_cast_fp8": (c_int, [P, c_int, c_long, P, c_int, P, P, P]),
    "pdt_cast_fp8_t": (c_int, [P, c_int, c_int, P, P, P]),
    "pdt_attn_bwd_q8": (c_int, [P] * 6 + [c_int, c_int, c_int, c_float] + [P] * 5),
    "pdt_attn_fwd_f8_q8": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P, P, P, P, P]),
    "pdt_cast_fp8_dual": (c_int, [P, c_int, c_int, P, P, P, P, P]),
    "pdt_fp8_meta_words": (c_int, []),
    "pdt_cast_fp8_delayed": (c_int, [P, c_int, c_long, P, c_int, P, P, P]),
    "pdt_fp8_meta_seed": (c_int, [P, c_long, c_int, P, P]),
    "pdt_attn_bwd": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_float, P]),
    "pdt_attn_bwd_f8": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_float, P]),
    "pdt_attn_bwd_f8_grid": (c_int, [c_int, c_int]),
    "pdt_attn_bwd_f8_q8": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_float, P, P, P, P, P, P, P]),
    "pdt_attn_set_pv8": (c_int, [c_int]),
    "pdt_attn_bwd_f8_debug": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_float, P, P]),
    "pdt_lenet_grad_row": (c_int, [c_int]),
    "pdt_lenet_fwd": (c_int, [P] * 9 + [c_int, c_int, c_int, c_float, c_float, c_uint, P, P, P, P]),
    "pdt_lenet_bwd": (c_int, [P] * 9 + [c_int, c_int, c_int, c_float, c_float, c_uint, P, P, P, P]),
    "pdt_nll_fwd": (c_int, [P, P, c_int, c_int, c_int, P, P, P, P]),
    "pdt_nll_bwd": (c_int, [P, P, P, c_int, c_int, c_int, P, P]),
}


def lib_path() -> Path:
    return _LIB_PATH


class OpTimer:
    """``PDT_OP_TIMING=1``: every launching entry point of the kernel library is bracketed
    by HIP events, and its device time attributed to (entry point, integer arguments) --
    the per-op, per-shape breakdown of a training step (scripts/op_profile.py). Query
    entry points (plans, row counts, workspace sizes) pass through untimed."""
    _QUERY = ("_rows", "_variants", "_plan", "_plan2", "_workspace", "_size", "_blocks", "_kind", "_resolve_variant",
              "_part", "_words", "_grad_row", "_set_unroll", "_set_bwd_single")

    def __init__(self, lib):
        self._lib = lib
        self.records = []
        self.enabled = False

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if not name.startswith("pdt_") or name.endswith(self._QUERY):
            return fn
        ints = [i for i, t in enumerate(_SIGS.get(name, (None, []))[1]) if t in (c_int, c_long, c_uint)]

        def call(*args):
            if not self.enabled or _capturing():
                return fn(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = fn(*args)
            e1.record()
            self.records.append((name, tuple(args[i] for i in ints if i < len(args)), e0, e1))
            return rc
        return call

    def summary(self, top=60):
        """[(ms, calls, name, int-args)] sorted by total time (synchronises)."""
        torch.cuda.synchronize()
        agg = {}
        for name, key, e0, e1 in self.records:
            ms = e0.elapsed_time(e1)
            ent = agg.setdefault((name, key), [0.0, 0])
            ent[0] += ms
            ent[1] += 1
        rows = sorted(((v[0], v[1], k[0], k[1]) for k, v in agg.items()), key=lambda r: -r[0])
        return rows[:top]


def _load():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not _LIB_PATH.exists():
                raise RuntimeError(f"native kernel library missing: {_LIB_PATH} -- run "
                                   "`python -m pytorch_distributed_template_amd.ops.build`")
            lib = ctypes.CDLL(str(_LIB_PATH))
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = OpTimer(lib) if os.environ.get("PDT_OP_TIMING", "0") == "1" else lib
    return _lib


def available() -> bool:
    if os.environ.get("PDT_DISABLE_NATIVE") == "1":
        return False
    return _LIB_PATH.exists() and torch.cuda.is_available()


def require():
    if not torch.cuda.is_available():
        raise RuntimeError("native HIP ops need a GPU")
    _load()


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_device = torch._C._cuda_getDevice


def _s():
    """The current HIP stream handle (the raw accessor: ~20x cheaper than
    ``torch.cuda.current_stream().cuda_stream``, which builds a Stream object per call)."""
    return _raw_stream(_cur_device())


def _p(t):
    return None if t is None else t.data_ptr()


def _chk(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


def _grad_buf(param, shape, memory_format=None, device=None):
    """fp32 output buffer for ``param``'s gradient: its slot in the data-parallel reducer's
    bucket when it has one (``parallel/reducer.py``: the kernel then writes the gradient where
    the all-reduce reads it, and autograd adopts that view as ``param.grad`` with no copy),
    else a new tensor of ``shape``."""
    if param is not None and getattr(param, "_pdt_grad_slot", None) is not None:
        from ..parallel.reducer import grad_out
        return grad_out(param, *shape, memory_format=memory_format)
    # no parameter (e.g. a bias gradient asked for without its bias tensor): the current GPU --
    # device=None would allocate on the HOST, and the kernel that fills the buffer would then
    # write through a host pointer (the illegal access of round 5's r5z variant sweep)
    dev = param.device if param is not None else device if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None)
    if memory_format is not None:
        return torch.empty(shape, dtype=torch.float32, device=dev, memory_format=memory_format)
    return torch.empty(shape, dtype=torch.float32, device=dev)


_FALLBACK_WARNED: set = set()


def fallback(what: str, reason: str) -> None:
    """Called where a native op cannot run its input and the stock PyTorch path would.
    Under backend ``native`` that is an error -- a run that asked for the HIP kernels
    never silently measures MIOpen / SDPA instead; under ``auto`` it warns once per op."""
    from . import fused
    if fused.get_backend() == "native":
        raise NotImplementedError(f"backend 'native': no HIP kernel path for {what} ({reason}); "
                                  "select backend 'auto' to allow the stock PyTorch op for it")
    if what not in _FALLBACK_WARNED:
        _FALLBACK_WARNED.add(what)
        import warnings
        warnings.warn(f"[pdt] {what}: {reason} -> stock PyTorch op", stacklevel=3)


def _cl(t: torch.Tensor) -> torch.Tensor:
    """channels_last-contiguous view/copy (NHWC storage)."""
    if t.dim() == 4 and not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    return t


def _empty_cl(n, c, h, w, dtype, device):
    return torch.empty((n, c, h, w), dtype=dtype, device=device, memory_format=torch.channels_last)


# =============================================================================
# bf16 weight shadows (cast once per parameter version)
# =============================================================================
_SHADOWS: dict = {}


def _same_tensor(ent_ref, w) -> bool:
    # id() and data_ptr() are both recycled after a tensor dies (a new Parameter of
    # the same size can get both): the cache entry must point at THIS object
    return ent_ref is not None and ent_ref() is w


def register_shadow(param: torch.Tensor, shadow: torch.Tensor):
    """Optimizers that write a bf16 copy while stepping register it here."""
    _SHADOWS[id(param)] = (shadow, param._version, param.data_ptr(), weakref.ref(param))


def bf16_weight(w: torch.Tensor, pad_cin_to: int | None = None) -> torch.Tensor:
    """bf16 copy of an fp32 weight in [Cout][..][Cin] (channels_last) storage."""
    if w.dtype == torch.bfloat16 and pad_cin_to is None:
        return _cl(w)
    key = (id(w), pad_cin_to)
    ent = _SHADOWS.get(key if pad_cin_to else id(w))
    if ent is not None and ent[1] == w._version and ent[2] == w.data_ptr() and _same_tensor(ent[3], w):
        return ent[0]
    src = _cl(w.detach())
    if pad_cin_to is not None and src.shape[1] != pad_cin_to:
        src = torch.nn.functional.pad(src, (0, 0, 0, 0, 0, pad_cin_to - src.shape[1]))
        src = _cl(src)
    out = torch.empty_like(src, dtype=torch.bfloat16, memory_format=torch.channels_last) if src.dim() == 4 \
        else torch.empty_like(src, dtype=torch.bfloat16)
    if src.dtype == torch.float32:
        _chk(_load().pdt_cast_f32_bf16(_p(src), _p(out), src.numel(), _s()), "cast")
    else:
        out.copy_(src)
    _SHADOWS[key if pad_cin_to else id(w)] = (out, w._version, w.data_ptr(), _weak(w))
    return out


def _weak(t):
    try:
        return weakref.ref(t)
    except TypeError:
        return None


# =============================================================================
# raw kernel wrappers
# =============================================================================
# -----------------------------------------------------------------------------
# Tile-variant autotuner: the first eager call of every distinct geometry times
# each tile variant (csrc/conv_igemm.hip, conv_wgrad.hip) with HIP events and
# keeps the fastest.
#   * The shipped table (_lib/autotune_gfx950.json, tracked) is READ-ONLY at run
#     time; new entries go to a per-user cache (PDT_AUTOTUNE_CACHE, default
#     ~/.cache/pytorch_distributed_template_amd/autotune_gfx950.json) overlaid
#     on it at load.
#   * PDT_AUTOTUNE=0 or --deterministic (PDT_DETERMINISTIC=1): no timing at all --
#     shipped/cached choices, else the fixed heuristic, so every run and every
#     rank picks the same variant (and the same split-K summation order).
#   * World size > 1: ranks must not time variants independently (different
#     choices per rank, stragglers inside the first backward). Tuning is off
#     unless :func:`pretune_distributed` runs: rank 0 tunes on one step and
#     broadcasts its table, then every rank freezes it.
# -----------------------------------------------------------------------------
_SHIPPED_TUNE_PATH = _LIB_PATH.parent / "autotune_gfx950.json"
_TUNE_PATH = Path(os.environ.get("PDT_AUTOTUNE_CACHE", str(Path.home() / ".cache" / "pytorch_distributed_template_amd"
                                                          / "autotune_gfx950.json")))
_TUNED: dict | None = None
_TUNE_FORCE = False   # pretune_distributed: rank 0 tunes although WORLD_SIZE > 1
_TUNE_FROZEN = False  # after the broadcast: no rank tunes any more


def _tuned() -> dict:
    global _TUNED
    if _TUNED is None:
        import json
        table = {}
        # PDT_AUTOTUNE_SHIPPED=0: ignore the shipped table (re-tuning experiments)
        paths = (_SHIPPED_TUNE_PATH, _TUNE_PATH) if os.environ.get("PDT_AUTOTUNE_SHIPPED", "1") != "0" \
            else (_TUNE_PATH,)
        for path in paths:
            try:
                table.update(json.loads(Path(path).read_text()))
            except Exception:
                pass
        _TUNED = table
    return _TUNED


def _save_tuned():
    """Persist the table to the user cache (never the installed package)."""
    if os.environ.get("RANK", "0") != "0" or _TUNE_PATH.resolve() == _SHIPPED_TUNE_PATH.resolve():
        return
    try:
        import json
        _TUNE_PATH.parent.mkdir(parents=True, exist_ok=True)
        tmp = str(_TUNE_PATH) + f".tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(_TUNED, f, indent=0, sort_keys=True)
        os.replace(tmp, _TUNE_PATH)
    except Exception:
        pass


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _tune_allowed() -> bool:
    if _TUNE_FROZEN or _capturing():
        return False
    if os.environ.get("PDT_AUTOTUNE", "1") == "0" or os.environ.get("PDT_DETERMINISTIC", "0") == "1":
        return False
    return _TUNE_FORCE or int(os.environ.get("WORLD_SIZE", "1")) <= 1


def pretune_distributed(run_step) -> None:
    """Agree on kernel variants across ranks before DDP training starts.

    ``run_step()`` runs one forward+backward on this rank's model (not yet
    DDP-wrapped). Rank 0 runs it with tuning enabled, then broadcasts its table;
    every rank adopts it and tuning is frozen (untuned shapes later fall back to
    the deterministic heuristic on every rank alike)."""
    global _TUNE_FORCE, _TUNE_FROZEN
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    obj = [None]
    if dist.get_rank() == 0:
        tune_on = os.environ.get("PDT_AUTOTUNE", "1") != "0" and os.environ.get("PDT_DETERMINISTIC", "0") != "1"
        err = None
        if tune_on:
            # the step must leave no trace on rank 0 that the other ranks do not share:
            # RNG streams are restored (DataLoader seeds, dropout), the fp8 scaling
            # histories it created or rolled are dropped (``_snapshot_fp8_meta``)
            cpu_rng = torch.get_rng_state()
            cuda_rng = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
            fp8_before = _snapshot_fp8_meta()
            _TUNE_FORCE = True
            try:
                run_step()
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
            except Exception as e:  # tell the other ranks instead of leaving them in the broadcast
                err = f"{type(e).__name__}: {e}"
            finally:
                _TUNE_FORCE = False
                torch.set_rng_state(cpu_rng)
                if cuda_rng is not None:
                    torch.cuda.set_rng_state(cuda_rng)
                _restore_fp8_meta(fp8_before)
        obj = [{"error": err} if err is not None else dict(_tuned())]
    dist.broadcast_object_list(obj, src=0)
    if isinstance(obj[0], dict) and set(obj[0]) == {"error"}:
        raise RuntimeError(f"kernel pre-tuning step failed on rank 0: {obj[0]['error']}")
    _tuned().clear()
    _tuned().update(obj[0])
    _TUNE_FROZEN = True


_FP8_META_ATTRS = ("_pdt_fp8_meta", "_pdt_fp8_gmeta")


def _snapshot_fp8_meta():
    """{module: {attr: clone}} of every live fp8 delayed-scaling state (nn.Linear owners)."""
    import gc
    snap = {}
    for obj in gc.get_objects():
        if isinstance(obj, nn.Module):
            st = {a: getattr(obj, a).clone() for a in _FP8_META_ATTRS if getattr(obj, a, None) is not None}
            snap[id(obj)] = (weakref.ref(obj), st)
    return snap


def _restore_fp8_meta(snap):
    """Undo what a step did to the fp8 scaling states: states it created are removed,
    states it rolled get their previous values back."""
    import gc
    for obj in gc.get_objects():
        if not isinstance(obj, nn.Module):
            continue
        ent = snap.get(id(obj))
        before = ent[1] if ent is not None and ent[0]() is obj else {}
        for a in _FP8_META_ATTRS:
            if getattr(obj, a, None) is None:
                continue
            if a in before:
                getattr(obj, a).copy_(before[a])
            else:
                delattr(obj, a)


NOT_APPLICABLE = -5  # kernel return code: this variant cannot run this geometry


class NotApplicable(RuntimeError):
    """An explicitly requested kernel variant cannot run this geometry / epilogue."""


def _chk_v(rc, name):
    if rc == NOT_APPLICABLE:
        raise NotApplicable(f"{name}: variant not applicable")
    _chk(rc, name)


def _time_variants(nvar, launch, allowed=None):
    """Fastest variant id: one warm launch each, then two interleaved rounds over all
    variants of a 3-launch HIP-event trial, best trial per variant (interleaving keeps a
    clock / cache transient from favouring whichever variants happen to run first)."""
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cand = []
    for v in range(nvar):
        if allowed is not None and v not in allowed:
            continue
        rc = launch(v)
        if rc == NOT_APPLICABLE:  # e.g. the streaming 1x1 kernel on a 3x3 geometry
            continue
        _chk(rc, f"tune variant {v}")
        cand.append(v)
    if not cand:
        return -1
    best_t = {v: float("inf") for v in cand}
    # PDT_TUNE_ROUNDS (default 2): interleaved rounds; more rounds cut the timing noise of a
    # (re)tune run at the cost of its length
    for _ in range(max(1, int(os.environ.get("PDT_TUNE_ROUNDS", "2")))):
        for v in cand:
            ev0.record()
            for _ in range(3):
                launch(v)
            ev1.record()
            ev1.synchronize()
            best_t[v] = min(best_t[v], ev0.elapsed_time(ev1))
    return min(cand, key=lambda v: best_t[v])


def _autotune(key, nvar, launch, default=0):
    table = _tuned()
    if key in table:
        return int(table[key])
    if not _tune_allowed():
        return default
    table[key] = _time_variants(nvar, launch)
    _save_tuned()
    return table[key]


def _id_set(spec):
    out = set()
    for part in spec.split(","):
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


def _variant_filter():
    """PDT_NT_VARIANTS="0-29,31" restricts the conv_nt variants the tuner may pick."""
    spec = os.environ.get("PDT_NT_VARIANTS")
    return _id_set(spec) if spec else None


_RETUNED: set = set()


def _retune_candidates(key, table):
    """PDT_RETUNE_WITH="45-48": a targeted re-tune of the table -- every conv_nt key already in
    it is timed once more against these new variant ids only (its current choice included),
    and switches when one of them is faster (PDT_RETUNE_PREFIX: only the keys of one family).
    Returns the allowed id set, or None (no re-tune)."""
    spec = os.environ.get("PDT_RETUNE_WITH")
    if not spec or key in _RETUNED or key not in table or not _tune_allowed():
        return None
    if not key.startswith(os.environ.get("PDT_RETUNE_PREFIX", "")):  # e.g. "ntb2:" (one key family)
        return None
    _RETUNED.add(key)
    return _id_set(spec) | {int(table[key])}


def _nt_args(src, b, out, stats, bias, a, act, variant, addend=None, aux=None, addend_mask=None):
    return (_p(src), _p(b), _p(out), _p(stats), _p(bias), _p(addend), _p(addend_mask), a["Hs"], a["Ws"], a["Cs"], a["Nimg"], a["Hm"], a["Wm"],
            a["Ncol"], a["K"], a["ldb"], a["sh"], a["sw"], a["oh0"], a["ow0"], a["dh"], a["dw"], a["nth"], a["ntw"],
            a["Ho"], a["Wo"], a["osh"], a["osw"], a["oph"], a["opw"], a["ldo"], int(act), _p(aux), int(variant),
            int(a.get("pix", 0)), _s())


# element-count limit of the unsigned 32-bit offsets in the A-staging BN apply (AX) and the fused
# BN-backward epilogue (csrc/conv_nt_tile.inc): ResNet-152 stage-1 activations at 3072 images per
# GPU (N x 56 x 56 x 256 = 2.47e9) are inside it; the rest of the conv path indexes in 64 bits
_AX_MAX_ELEMS = 2 ** 32 - 8


def _check_nt(src, b, out, a):
    assert src.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and out.dtype == torch.bfloat16
    Cs, K, Ncol, ldo, ldb = a["Cs"], a["K"], a["Ncol"], a["ldo"], a["ldb"]
    assert Cs % 8 == 0 and K % 8 == 0 and Ncol % 8 == 0 and ldo % 8 == 0, (Cs, K, Ncol, ldo)
    assert K == a["nth"] * a["ntw"] * Cs
    # bounds: the kernel reads src[0 : Nimg*Hs*Ws*Cs], b[0 : Ncol*ldb], writes out rows < Nimg*Ho*Wo
    pix = a.get("pix", 0) or Cs  # elements per source pixel in memory
    assert pix % 4 == 0 and pix <= Cs
    assert src.numel() >= a["Nimg"] * a["Hs"] * a["Ws"] * pix, "src too small"
    assert b.numel() >= Ncol * ldb or K == 0, "B too small"
    assert out.numel() >= a["Nimg"] * a["Ho"] * a["Wo"] * ldo, "out too small"
    assert a["Hm"] * a["osh"] <= a["Ho"] and a["Wm"] * a["osw"] <= a["Wo"]
    # pixel indices are 32-bit; element offsets are 64-bit except the A-staging BN apply and the
    # BN-backward epilogue, which use unsigned 32-bit offsets (limit _AX_MAX_ELEMS, checked by the
    # library: it refuses those paths beyond it)
    assert a["Nimg"] * a["Hs"] * a["Ws"] < 2 ** 31 and a["Nimg"] * a["Ho"] * a["Wo"] < 2 ** 31


_NT_KEYS: dict = {}  # geometry tuple -> tuned-table key string (built once per geometry)


def select_nt_variant(src, b, out, *, with_stats=False, bias=None, act=0, aux=None, addend=None, **a):
    """Variant id for this geometry and epilogue (tuning it on first use when allowed)."""
    M = a["Nimg"] * a["Hm"] * a["Wm"]
    geom = (a["Hs"], a["Ws"], a["Cs"], a["Nimg"], a["Hm"], a["Wm"], a["Ncol"], a["K"], a["sh"], a["sw"], a["nth"],
            a["ntw"], a["osh"], int(with_stats), int(bias is not None), a.get("pix", 0), int(act))
    key = _NT_KEYS.get(geom)
    if key is None:
        key = "nt5:" + ",".join(str(x) for x in geom[:15])
        if a.get("pix"):
            key += f",p{a['pix']}"
        if act:  # epilogue work changes the best tile (and the streaming 1x1 kernels take no activation)
            key += f",a{int(act)}"
        _NT_KEYS[geom] = key
    table = _tuned()
    allowed = _retune_candidates(key, table)
    if key in table and allowed is None:
        return int(table[key])
    lib = _load()
    if not _tune_allowed():
        return lib.pdt_conv_nt_resolve_variant(-1, M, a["Ncol"], a["K"])
    _check_nt(src, b, out, a)
    nvar = lib.pdt_conv_nt_num_variants()
    # partial-stat rows depend on the variant's BM and waves-along-M: size for the largest
    rows = max(lib.pdt_conv_nt_stat_rows(M, a["Ncol"], a["K"], v) for v in range(nvar))
    stats = torch.empty(2 * rows * a["Ncol"], dtype=torch.float32, device=src.device) if with_stats else None
    tune_add = addend if act in (3, 5) else None  # acts 3 / 5 read their operand through the addend pointer
    best = _time_variants(nvar, lambda v: lib.pdt_conv_nt(*_nt_args(src, b, out, stats, bias, a, act, v, aux=aux,
                                                                    addend=tune_add)),
                          allowed if allowed is not None else _variant_filter())
    table[key] = best
    _save_tuned()
    return best


ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2}
# epilogue ids beyond ACT: 3 = out * gelu'(addend = z); 4 = GELU whose aux output is gelu'(z)
# (not z) -- both from one tanh; 5 = out * addend (the stored derivative)
ACT_GELU_GRAD, ACT_GELU_DUAL, ACT_MUL = 3, 4, 5


def _gelu_dual() -> bool:
    """The MLP stores gelu'(z) in the fc1 epilogue (act 4) and its backward multiplies by it
    in the fc2 data-gradient epilogue (act 5) -- the derivative's tanh is not recomputed there.
    PDT_GELU_DUAL=0: store z and recompute gelu'(z) in the backward epilogue (acts 2 / 3)."""
    return os.environ.get("PDT_GELU_DUAL", "1") == "1"


def conv_nt(src, b, out, *, stats=None, bias=None, relu=False, act=None, variant=None, addend=None, aux=None,
            addend_mask=None, **a):
    """C[m, n] = sum_k A[m, k] B[n, k] (+ addend) with the implicit-GEMM gather (see csrc/conv_igemm.hip)."""
    _check_nt(src, b, out, a)
    if addend is not None:
        assert addend.dtype == torch.bfloat16 and addend.numel() == out.numel() and addend.is_contiguous(
            memory_format=torch.channels_last if addend.dim() == 4 else torch.contiguous_format)
    act_id = (act if isinstance(act, int) else ACT[act]) if act is not None else (1 if relu else 0)
    if aux is not None:
        assert aux.dtype == torch.bfloat16 and aux.numel() == out.numel()
    if variant is None:
        variant = select_nt_variant(src, b, out, with_stats=stats is not None, bias=bias, act=act_id, aux=aux,
                                    addend=addend, **a)
    if addend_mask is not None:
        assert addend is not None and addend_mask.dtype == torch.uint8 and addend_mask.numel() * 8 == addend.numel()
        assert a["ldo"] == a["Ncol"]
    lib = _load()
    rc = lib.pdt_conv_nt(*_nt_args(src, b, out, stats, bias, a, act_id, variant, addend, aux, addend_mask))
    if rc == NOT_APPLICABLE:  # a cached variant tuned for another epilogue (e.g. the streaming 1x1 kernel)
        M = a["Nimg"] * a["Hm"] * a["Wm"]
        variant = lib.pdt_conv_nt_resolve_variant(-1, M, a["Ncol"], a["K"])
        rc = lib.pdt_conv_nt(*_nt_args(src, b, out, stats, bias, a, act_id, variant, addend, aux, addend_mask))
    _chk(rc, "conv_nt")


def _check_addend(addend, out, addend_mask, Ncol):
    assert addend.dtype == torch.bfloat16 and addend.numel() == out.numel() and addend.is_contiguous(
        memory_format=torch.channels_last if addend.dim() == 4 else torch.contiguous_format)
    if addend_mask is not None:
        assert addend_mask.dtype == torch.uint8 and addend_mask.numel() * 8 == addend.numel()


def conv_stat_rows(M, Ncol, K, variant):
    return _load().pdt_conv_nt_stat_rows(M, Ncol, K, variant)


def _wgrad_launch(lib, dy, x, out, v, scale, accumulate, a, bias_out=None, bna=None):
    """One weight-gradient launch (+ slab reduction); returns the kernel's return code
    (NOT_APPLICABLE: variant ``v`` cannot run this geometry). ``bna`` = (y, coef [5][Mo]):
    ``dy`` is dA and the BN backward apply runs in the dY staging (``pdt_conv_wgrad2``)."""
    kps = c_int(0)
    splits = lib.pdt_wgrad_plan2(a["M"], a["Mo"], a["No"], a["Hs"], a["Ws"], a["C"], v, ctypes.byref(kps))
    if splits < 0:
        return splits
    slab = torch.empty(lib.pdt_wgrad_workspace(splits, a["Mo"], a["No"]), dtype=torch.float32, device=dy.device)
    by, bc = bna if bna is not None else (None, None)
    return lib.pdt_conv_wgrad2(_p(dy), _p(x), _p(slab), _p(out), a["M"], a["Mo"], a["No"], a["ldy"], a["Hs"],
                               a["Ws"], a["C"], a["Hm"], a["Wm"], a["sh"], a["sw"], a["oh0"], a["ow0"], a["dh"],
                               a["dw"], a["ntw"], splits, kps.value, float(scale), int(accumulate), int(v),
                               int(a.get("pix", 0)), _p(bias_out), _p(by), _p(bc), _s())


WGB_VARIANTS = tuple(range(12))  # the 4-wave 1/2-stage tiles carry the BN-apply instantiation


def conv_wgrad_bn(dA, x, out, y, coef, run_ref, **a):
    """Weight gradient whose dY = k1*gate(dA) + k2*y + k3 (a BN+ReLU unit's backward apply,
    ``coef`` = [k1; k2; k3; scale; shift] fp32 [5][Mo], gate = y*scale+shift > 0) is formed
    while staging dA (``pdt_conv_wgrad2``): the apply pass and its dy tensor disappear.
    Tuned per geometry against ``run_ref()`` (the element pass + the plain weight gradient):
    returns False when that is faster (the caller runs it), True when done here."""
    lib = _load()
    assert coef.dtype == torch.float32 and coef.is_contiguous() and coef.numel() == 5 * a["Mo"]
    assert y.dtype == torch.bfloat16 and y.shape == dA.shape
    key = "wgb:" + ",".join(str(a[k]) for k in ("M", "Mo", "No", "Hs", "Ws", "C", "Hm", "Wm", "sh", "ntw")) + \
        (f",p{a['pix']}" if a.get("pix") else "")
    table = _tuned()
    v = table.get(key)
    if v is None:
        if not _tune_allowed():
            return False

        def run(v):
            return _wgrad_launch(lib, dA, x, out, v, 1.0, False, a, bna=(y, coef))
        best = _time_variants(max(WGB_VARIANTS) + 1, run, set(WGB_VARIANTS))
        if best >= 0 and _time_fn(run_ref) < _time_fn(lambda: run(best)):
            best = AX_UNFUSED
        table[key] = v = best
        _save_tuned()
    v = int(v)
    if v < 0:
        return False
    _chk(_wgrad_launch(lib, dA, x, out, v, 1.0, False, a, bna=(y, coef)), "conv_wgrad (BN backward apply)")
    return True


_WG_KEYS: dict = {}


def conv_wgrad(dy, x, out, *, scale=1.0, accumulate=False, variant=None, bias_out=None, **a):
    """dW[co, tap*C + c] = sum_m dY[m, co] X_gather[m, (tap, c)] (see csrc/conv_wgrad.hip).
    ``bias_out`` (fp32 [Mo]): also sum_m dY[m, co] -- the nn.Linear bias gradient -- from the
    dY tiles the kernel stages anyway (no separate column-sum pass)."""
    M, Mo, No, ldy, C, Hm, Wm = a["M"], a["Mo"], a["No"], a["ldy"], a["C"], a["Hm"], a["Wm"]
    assert dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and out.dtype == torch.float32
    assert C % 8 == 0 and Mo % 8 == 0 and No % 8 == 0 and ldy % 8 == 0
    assert out.numel() >= Mo * No and dy.numel() >= M * ldy
    pix = a.get("pix", 0) or C  # elements per source pixel in memory
    assert pix % 4 == 0 and pix <= C
    assert M % (Hm * Wm) == 0 and x.numel() >= (M // (Hm * Wm)) * a["Hs"] * a["Ws"] * pix, "wgrad source too small"
    assert a["ntw"] >= 1 and No % C == 0
    if bias_out is not None:
        assert bias_out.dtype == torch.float32 and bias_out.numel() >= Mo and bias_out.is_contiguous()
        assert bias_out.device == dy.device, "bias gradient buffer on another device than dY"
    assert out.device == dy.device == x.device, "weight gradient operands on different devices"
    lib = _load()
    if variant is None:
        gt = (a["M"], a["Mo"], a["No"], a["Hs"], a["Ws"], a["C"], a["Hm"], a["Wm"], a["sh"], a["ntw"], a.get("pix", 0))
        key = _WG_KEYS.get(gt)
        if key is None:
            key = "wg2:" + ",".join(str(x) for x in gt[:10])
            if a.get("pix"):
                key += f",p{a['pix']}"
            _WG_KEYS[gt] = key
        table = _tuned()
        spec = os.environ.get("PDT_RETUNE_WG")  # targeted re-tune of shipped keys against these ids
        if key in table and spec and key not in _RETUNED and _tune_allowed():
            _RETUNED.add(key)
            allowed = _id_set(spec) | {int(table[key])}
            table[key] = _time_variants(lib.pdt_wgrad_num_variants(),
                                        lambda v: _wgrad_launch(lib, dy, x, out, v, scale, False, a), allowed)
            _save_tuned()
        if key in table:
            variant = int(table[key])
        elif not _tune_allowed():
            variant = -1
        else:
            best = _time_variants(lib.pdt_wgrad_num_variants(),
                                  lambda v: _wgrad_launch(lib, dy, x, out, v, scale, False, a))
            table[key] = best
            _save_tuned()
            variant = best
    rc = _wgrad_launch(lib, dy, x, out, variant, scale, accumulate, a, bias_out)
    if rc == NOT_APPLICABLE:  # e.g. a tuned halo id for a geometry it does not cover: the heuristic tile
        rc = _wgrad_launch(lib, dy, x, out, -1, scale, accumulate, a, bias_out)
    _chk(rc, "conv_wgrad")


def colsum(x, R, C):
    """fp32 column sums of a bf16 [R][C] matrix (bias gradients)."""
    assert x.dtype == torch.bfloat16 and x.numel() >= R * C
    lib = _load()
    out = torch.empty(C, dtype=torch.float32, device=x.device)
    work = torch.empty(lib.pdt_colsum_workspace(R, C), dtype=torch.float32, device=x.device)
    _chk(lib.pdt_colsum(_p(x), _p(out), _p(work), R, C, 0, _s()), "colsum")
    return out


def fill_uniform_(t: torch.Tensor, seed: int):
    assert t.dtype == torch.bfloat16 and t.numel() % 8 == 0
    _chk(_load().pdt_fill_uniform_bf16(_p(t), t.numel(), seed & 0xFFFFFFFF, _s()), "fill")
    return t


def synthetic_images_at(buf, idx, C, seed, labels, num_classes):
    """Samples ``idx`` (int64 [B], device) of the index-addressable synthetic dataset into
    ``buf`` (bf16 [B, H, W, Cp], channels >= C zeroed) and ``labels`` (int64 [B])."""
    B, H, W, Cp = buf.shape
    assert buf.dtype == torch.bfloat16 and buf.is_contiguous() and Cp % 4 == 0 and C <= Cp
    assert idx.dtype == torch.int64 and idx.numel() == B and idx.device == buf.device
    assert labels.dtype == torch.int64 and labels.numel() == B and labels.device == buf.device
    _chk(_load().pdt_synth_images_bf16(_p(buf), _p(idx), B, H * W, C, Cp, seed & 0xFFFFFFFF, _p(labels),
                                       int(num_classes), _s()), "synth_images")


def synthetic_images(shape, dtype, device, seed=0, channels_last=True):
    n, c, h, w = shape
    if channels_last:
        x = torch.empty(shape, dtype=torch.bfloat16, device=device, memory_format=torch.channels_last)
    else:
        x = torch.empty(shape, dtype=torch.bfloat16, device=device)
    fill_uniform_(x, seed)
    return x if dtype == torch.bfloat16 else x.to(dtype)


# =============================================================================
# conv geometry helpers
# =============================================================================
def _fwd_geom(N, H, W, Cs, conv: nn.Conv2d):
    KH, KW = conv.kernel_size
    sh, sw = conv.stride
    ph, pw = conv.padding
    Ho = (H + 2 * ph - KH) // sh + 1
    Wo = (W + 2 * pw - KW) // sw + 1
    return dict(KH=KH, KW=KW, sh=sh, sw=sw, ph=ph, pw=pw, Ho=Ho, Wo=Wo)


def supports_conv(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    if conv.groups != 1 or conv.dilation != (1, 1) or conv.bias is not None:
        return False
    if x.dim() != 4 or conv.out_channels % 8 != 0:
        return False
    N, C, H, W = x.shape
    if C % 8 != 0 and C > 8:
        return False
    sh, sw = conv.stride
    if (H % sh) or (W % sw):
        return False
    return True


def _fwd_nt_geom(N, H, W, Cs, Cout, g):
    K = g["KH"] * g["KW"] * Cs
    return dict(Hs=H, Ws=W, Cs=Cs, Nimg=N, Hm=g["Ho"], Wm=g["Wo"], Ncol=Cout, K=K, ldb=K, sh=g["sh"], sw=g["sw"],
                oh0=-g["ph"], ow0=-g["pw"], dh=1, dw=1, nth=g["KH"], ntw=g["KW"], Ho=g["Ho"], Wo=g["Wo"], osh=1,
                osw=1, oph=0, opw=0, ldo=Cout)


def _conv_forward(x, wb, N, H, W, Cs, Cout, g, with_stats=False):
    """Forward conv; returns (y, M, stats_partials or None, stats_rows)."""
    M = N * g["Ho"] * g["Wo"]
    y = _empty_cl(N, Cout, g["Ho"], g["Wo"], torch.bfloat16, x.device)
    a = _fwd_nt_geom(N, H, W, Cs, Cout, g)
    v = select_nt_variant(x, wb, y, with_stats=with_stats, **a)
    part, R = None, 0
    if with_stats:
        lib = _load()
        R = conv_stat_rows(M, Cout, a["K"], v)
        part = torch.empty(2 * R * Cout + lib.pdt_rows_reduce_workspace(R, Cout), dtype=torch.float32,
                           device=x.device)
    conv_nt(x, wb, y, stats=part, variant=v, **a)
    return y, M, part, R


class _DgradWeights:
    """Cache of the transposed, stride-phase-sliced bf16 weights the dgrad GEMMs
    consume (pdt_wt_dgrad layout), keyed per (parameter, phase). When the
    optimizer has stepped (parameter version changed), the FIRST request
    rebuilds every registered entry in ONE multi-tensor launch
    (pdt_wt_dgrad_multi) instead of one small kernel per conv and phase."""

    def __init__(self):
        self.entries = {}   # key -> [weakref(param), buf, version, job-tuple, data_ptr]
        self.table = None   # device job table (uint8) for the current entry set
        self.total = 0

    def get(self, param, Cout, KH, KW, Cin, kh0, kw0, s, nth, ntw):
        key = (id(param), param.data_ptr(), kh0, kw0, s, nth, ntw)
        ent = self.entries.get(key)
        if ent is not None and ent[0]() is param and ent[2] == param._version:
            return ent[1]
        lib = _load()
        if (ent is None or ent[0]() is not param) and len(self.entries) >= 512:
            self.entries.clear()  # device job table holds at most 512 entries
            self.table = None
        if ent is None or ent[0]() is not param:
            import weakref
            buf = torch.empty(max(Cin * nth * ntw * Cout, 8), dtype=torch.bfloat16, device=param.device)
            _chk(lib.pdt_wt_dgrad(_p(param), _p(buf), Cout, KH, KW, Cin, kh0, kw0, s, nth, ntw, _s()), "wt_dgrad")
            self.entries[key] = [weakref.ref(param), buf, param._version, (Cout, KH, KW, Cin, kh0, kw0, s, nth, ntw),
                                 param.data_ptr()]
            self.table = None
            return buf
        self._rebuild_all(lib)
        return ent[1]

    def _rebuild_all(self, lib):
        # drop entries whose parameter died or moved (their pointers must never reach the kernel)
        dead = [k for k, e in self.entries.items() if e[0]() is None or e[0]().data_ptr() != e[4]]
        for k in dead:
            del self.entries[k]
            self.table = None
        if self.table is None:
            import struct
            assert lib.pdt_wt_job_size() == 64
            blob, start = bytearray(), 0
            for ref, buf, _, j, ptr in self.entries.values():
                blob += struct.pack("<QQq10i", ptr, buf.data_ptr(), start, *j, 0)
                start += j[3] * j[7] * j[8] * j[0]
            dev = next(iter(self.entries.values()))[1].device
            self.table = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
            self.total = start
        _chk(lib.pdt_wt_dgrad_multi(_p(self.table), len(self.entries), self.total, _s()), "wt_dgrad_multi")
        for ent in self.entries.values():
            ent[2] = ent[0]()._version


_DGRAD_W = _DgradWeights()


class _BnbPartials:
    """BatchNorm-backward partial sums produced by a data-gradient epilogue for one
    unit (see ``BnbArgs`` in csrc/conv_igemm.hip): [2][R][C] fp32 (+ rows_reduce tail).
    ``second``: the same epilogue's partials for a second unit fed by the same gated
    gradient (a downsample block's shortcut BN), or None."""
    __slots__ = ("part", "R", "unit", "second")

    def __init__(self, part, R, unit, second=None):
        self.part, self.R, self.unit, self.second = part, R, unit, second


def _bnb_enabled() -> bool:
    return os.environ.get("PDT_FUSE_BN_BWD", "1") != "0"


def _bnb2_enabled() -> bool:
    """A downsample block's shortcut-BN backward partials in the next block's data-gradient
    epilogue (PDT_FUSE_BN_BWD2=0: its own reduce pass over dout and the shortcut output)."""
    return os.environ.get("PDT_FUSE_BN_BWD2", "1") != "0"


def _conv_dgrad(dy, w32, N, H, W, Cin, Cout, g, addend=None, addend_mask=None, bnb_unit=None, bnb_mask=None,
                bnb_unit2=None):
    """dX [N,Cin,H,W] (+ addend) from dY [N,Cout,Ho,Wo] (stride phases, see csrc/conv_igemm.hip).

    ``bnb_unit``: the conv->BN(->ReLU) unit whose output dX is the gradient of; its
    BatchNorm-backward reduction (gated by its ReLU -- ``bnb_mask`` or recomputed
    from y) is computed in the GEMM epilogue. Returns ``(dx, _BnbPartials)`` then.
    ``bnb_unit2``: a second unit fed by the same gated gradient (``bnb_mask`` required),
    whose partials the same epilogue also produces (``_BnbPartials.second``; None where
    the tuned tile cannot)."""
    KH, KW, s_h, s_w, ph, pw = g["KH"], g["KW"], g["sh"], g["sw"], g["ph"], g["pw"]
    assert w32.shape[0] == Cout and w32.shape[1] == Cin, (tuple(w32.shape), Cout, Cin)
    assert dy.shape[1] == Cout and dy.numel() == N * Cout * g["Ho"] * g["Wo"]
    dx = _empty_cl(N, Cin, H, W, torch.bfloat16, dy.device)
    lib = _load()
    # parameters (fp32, channels_last storage) get cached phase weights; temporaries do not
    cacheable = isinstance(w32, nn.Parameter) and w32.dtype == torch.float32 and \
        w32.is_contiguous(memory_format=torch.channels_last)
    w32c = w32 if cacheable else _cl(w32.detach().float())
    launches = []
    for qh in range(s_h):
        kh0 = (qh + ph) % s_h
        nth = (KH - kh0 + s_h - 1) // s_h if kh0 < KH else 0
        oh0 = (qh + ph - kh0) // s_h
        for qw in range(s_w):
            kw0 = (qw + pw) % s_w
            ntw = (KW - kw0 + s_w - 1) // s_w if kw0 < KW else 0
            ow0 = (qw + pw - kw0) // s_w
            K = nth * ntw * Cout
            assert s_h == s_w, "dgrad weight slicing assumes square strides"
            if K > 0 and cacheable:
                wt = _DGRAD_W.get(w32, Cout, KH, KW, Cin, kh0, kw0, s_h, nth, ntw)
            else:
                wt = torch.empty(max(Cin * K, 8), dtype=torch.bfloat16, device=dy.device)
                if K > 0:
                    _chk(lib.pdt_wt_dgrad(_p(w32c), _p(wt), Cout, KH, KW, Cin, kh0, kw0, s_h, nth, ntw, _s()),
                         "wt_dgrad")
            a = dict(Hs=g["Ho"], Ws=g["Wo"], Cs=Cout, Nimg=N, Hm=H // s_h, Wm=W // s_w, Ncol=Cin,
                     K=K, ldb=max(K, 8), sh=1, sw=1, oh0=oh0, ow0=ow0, dh=-1, dw=-1, nth=nth, ntw=max(ntw, 0),
                     Ho=H, Wo=W, osh=s_h, osw=s_w, oph=qh, opw=qw, ldo=Cin)
            if bnb_unit is None:
                conv_nt(dy, wt, dx, addend=addend, addend_mask=addend_mask, **a)
            else:
                launches.append((wt, a))
    if bnb_unit is None:
        return dx
    # fused BN-backward partials: every phase launch writes its own row range
    u = bnb_unit
    assert u.Cout == Cin and u.y.numel() == dx.numel() and u.y.is_contiguous(memory_format=torch.channels_last)
    if addend is not None:
        _check_addend(addend, dx, addend_mask, Cin)
    relu = bool(u.relu or bnb_mask is not None)
    if bnb_mask is not None:
        assert bnb_mask.dtype == torch.uint8 and bnb_mask.numel() * 8 == dx.numel()

    def launch(wt, a, v, part, row0, R, part2=None):
        args = (_p(dy), _p(wt), _p(dx), _p(addend), _p(addend_mask), a["Hs"], a["Ws"], a["Cs"], a["Nimg"], a["Hm"],
                a["Wm"], a["Ncol"], a["K"], a["ldb"], a["sh"], a["sw"], a["oh0"], a["ow0"], a["dh"], a["dw"], a["nth"],
                a["ntw"], a["Ho"], a["Wo"], a["osh"], a["osw"], a["oph"], a["opw"], a["ldo"], int(v), _p(u.y),
                _p(u.mean), _p(u.scale), _p(u.shift), _p(bnb_mask), _p(part), int(relu), int(row0), int(R))
        if part2 is None:
            return lib.pdt_conv_nt_bnb(*args, _s())
        return lib.pdt_conv_nt_bnb2(*args, _p(u2.y), _p(u2.mean), _p(part2), _s())

    u2 = bnb_unit2
    if u2 is not None and (bnb_mask is None or u2.Cout != Cin or u2.y.shape != u.y.shape or
                           not u2.y.is_contiguous(memory_format=torch.channels_last)):
        u2 = None
    plan, R = [], 0
    has_add, has_mask = int(addend is not None), int(bnb_mask is not None)
    for wt, a in launches:
        _check_nt(dy, wt, dx, a)
        # with a second unit the tile is tuned with its partials (own key: the ring tiles cannot)
        v = _select_bnb_variant(lambda v, part, rows, part2, wt=wt, a=a: launch(wt, a, v, part, 0, rows, part2), a,
                                addend is not None, bnb_mask is not None, dy.device, two=u2 is not None)
        # a table / heuristic choice whose epilogue does not compile this configuration (a ring
        # tile): without the second unit if that is all it lacks, else the generic 64x128 tile
        if not lib.pdt_conv_nt_bnb_supports(v, has_add, has_mask, int(relu), int(u2 is not None)):
            if u2 is not None and lib.pdt_conv_nt_bnb_supports(v, has_add, has_mask, int(relu), 0):
                u2 = None
            else:
                v = _BNB_GENERIC_VARIANT
        rows = lib.pdt_conv_nt_bnb_rows(a["Nimg"] * a["Hm"] * a["Wm"], Cin, a["K"], v)
        plan.append((wt, a, v, R))
        R += rows
    one = 2 * R * Cin + lib.pdt_rows_reduce_workspace(R, Cin)
    if u2 is None:
        part = torch.empty(one, dtype=torch.float32, device=dy.device)
        for wt, a, v, row0 in plan:
            _chk(launch(wt, a, v, part, row0, R), "conv_nt_bnb")
        return dx, _BnbPartials(part, R, u)
    # both units' [2][R][C] blocks (+ their reduce tails) in one buffer, the second 256-B aligned
    off = (one + 63) // 64 * 64
    buf = torch.empty(off + one, dtype=torch.float32, device=dy.device)
    part, part2 = buf[:one], buf[off:]
    second = True
    for wt, a, v, row0 in plan:
        rc = launch(wt, a, v, part, row0, R, part2 if second else None)
        if rc == NOT_APPLICABLE and second:  # tuned tile without the second-unit epilogue
            second = False
            for wt_, a_, v_, row0_ in plan:  # redo every phase launch without it
                _chk(launch(wt_, a_, v_, part, row0_, R), "conv_nt_bnb")
            break
        _chk(rc, "conv_nt_bnb2")
    return dx, _BnbPartials(part, R, u, _BnbPartials(part2, R, u2) if second else None)


_NTB_KEYS: dict = {}
_BNB_GENERIC_VARIANT = 17  # 64x128 LDS tile, direct store: every BN-backward epilogue configuration


def _select_bnb_variant(launch, a, has_addend, has_mask, device, two=False):
    """Variant for a data gradient with the fused BN-backward epilogue: its own
    tuned-table key (the epilogue's extra loads / registers shift the best tile);
    ``two``: also a second unit's partials (key suffix ",2", timed with them)."""
    gt = (a["Hs"], a["Ws"], a["Cs"], a["Nimg"], a["Hm"], a["Wm"], a["Ncol"], a["K"], a["sh"], a["sw"], a["nth"],
          a["ntw"], a["osh"], int(has_addend), int(has_mask)) + ((2,) if two else ())
    key = _NTB_KEYS.get(gt)
    if key is None:
        key = _NTB_KEYS[gt] = "ntb2:" + ",".join(str(x) for x in gt)
    geom = ",".join(str(x) for x in gt[:13])
    table = _tuned()
    allowed = _retune_candidates(key, table)
    if key in table and allowed is None:
        return int(table[key])
    lib = _load()
    M = a["Nimg"] * a["Hm"] * a["Wm"]
    if not _tune_allowed():  # the plain data gradient's tuned tile, else the heuristic
        plain = f"nt5:{geom},0,0"
        return int(table[plain]) if plain in table else lib.pdt_conv_nt_resolve_variant(-1, M, a["Ncol"], a["K"])
    nvar = lib.pdt_conv_nt_num_variants()
    rows = max(lib.pdt_conv_nt_bnb_rows(M, a["Ncol"], a["K"], v) for v in range(nvar))
    part = torch.empty(2 * rows * a["Ncol"], dtype=torch.float32, device=device)
    part2 = torch.empty_like(part) if two else None
    table[key] = _time_variants(nvar, lambda v: launch(v, part, lib.pdt_conv_nt_bnb_rows(M, a["Ncol"], a["K"], v),
                                                       part2),
                                allowed if allowed is not None else _variant_filter())
    _save_tuned()
    return table[key]


def _conv_wgrad(dy, x, N, H, W, Cs, Cout, g, out):
    M = N * g["Ho"] * g["Wo"]
    conv_wgrad(dy, x, out, M=M, Mo=Cout, No=g["KH"] * g["KW"] * Cs, ldy=Cout, Hs=H, Ws=W, C=Cs, Hm=g["Ho"],
               Wm=g["Wo"], sh=g["sh"], sw=g["sw"], oh0=-g["ph"], ow0=-g["pw"], dh=1, dw=1, ntw=g["KW"])


# =============================================================================
# fused conv -> BN -> (+res) -> (ReLU): one "unit"
# =============================================================================
class _BNArgs:
    """BatchNorm module state resolved for one call (training vs eval, running
    stats, num_batches_tracked handled inside the finalize kernel)."""
    __slots__ = ("training", "momentum", "eps", "rm", "rv", "nbt")

    def __init__(self, bn: nn.BatchNorm2d):
        self.training = bn.training or not bn.track_running_stats
        self.momentum = bn.momentum if bn.momentum is not None else 0.1
        self.eps = bn.eps
        self.rm = bn.running_mean if (bn.track_running_stats and bn.training) else None
        self.rv = bn.running_var if (bn.track_running_stats and bn.training) else None
        self.nbt = None
        if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
            self.nbt = bn.num_batches_tracked
            if bn.momentum is None:  # cumulative moving average needs the host-side count
                self.nbt.add_(1)
                self.momentum = 1.0 / float(self.nbt.item())
                self.nbt = None
        if not self.training:
            self.rm, self.rv = bn.running_mean, bn.running_var


class _Unit:
    """Saved state of one conv->BN->act unit between forward and backward."""
    __slots__ = ("x", "w", "gamma", "beta", "y", "act", "mask", "mean", "invstd", "scale", "shift", "N", "C", "Cs", "H",
                 "W", "Cout", "g", "relu", "has_res", "bnb_pre", "pend", "res_unit", "__weakref__")


def nhwc_padded_view(x, cp):
    """[N, cp, H, W] channels_last view of a [N, C, H, W] bf16 tensor that a loader
    built as a view into NHWC storage zero-padded to ``cp`` channels
    (``x.pdt_nhwc_pad == cp``); None when x is not such a view."""
    if getattr(x, "pdt_nhwc_pad", None) != cp or x.dtype != torch.bfloat16 or x.dim() != 4:
        return None
    N, C, H, W = x.shape
    if x.stride() != (H * W * cp, 1, W * cp, cp):
        return None
    if x.untyped_storage().nbytes() < (x.storage_offset() + N * H * W * cp) * 2:
        return None
    return torch.as_strided(x, (N, cp, H, W), (H * W * cp, 1, W * cp, cp))


def _unit_fwd(x, w, gamma, beta, residual, conv, relu, bna: _BNArgs, apply: bool = True, res_unit=None,
              src_pend=None, defer: bool = False):
    """conv -> BN (batch statistics from the conv epilogue) -> (+ residual) -> (ReLU).
    ``res_unit``: the residual is that unit's RAW conv output and its BN affine is applied
    inside this unit's BN apply (``residual`` must be ``res_unit.y``).
    ``defer``: skip the BN(+res)+ReLU element pass; the returned output buffer is still
    unwritten (``u.pend`` set) and the NEXT unit that reads it must be called with
    ``src_pend=u`` -- its 1x1 GEMM computes the apply in its A staging and writes the
    buffer (+ ReLU mask) once (``_conv_fwd_ax``), or the element pass runs first."""
    lib = _load()
    st = _s()
    N, C, H, W = x.shape
    Cs = C if C % 8 == 0 else 8
    xp = nhwc_padded_view(x, Cs) if Cs != C else None
    x = x.to(torch.bfloat16)
    if xp is not None:  # stem on a loader-padded NHWC batch: read in place
        x = xp
    elif Cs != C:  # stem: pad channels to 8 (NHWC)
        x = torch.nn.functional.pad(_cl(x).permute(0, 2, 3, 1), (0, Cs - C)).permute(0, 3, 1, 2)
    x = _cl(x)
    Cout = w.shape[0]
    g = _fwd_geom(N, H, W, Cs, conv)
    wb = bf16_weight(w, pad_cin_to=Cs if Cs != C else None)
    f32 = dict(dtype=torch.float32, device=x.device)
    M = N * g["Ho"] * g["Wo"]
    r = None
    if src_pend is not None and getattr(src_pend, "pend", None) is not None:
        assert src_pend.y.shape == x.shape and x.data_ptr() == src_pend.pend[2].data_ptr()
        r = _conv_fwd_ax(src_pend, x, wb, N, H, W, Cs, Cout, g, bna.training)
        if r is None:  # not covered by the AX tiles: the deferred element pass, then the plain GEMM
            _materialize(src_pend)
        src_pend.pend = None
    if r is None:
        r = _conv_forward(x, wb, N, H, W, Cs, Cout, g, with_stats=bna.training)
    y, _, part, R = r
    if bna.training:
        vec = torch.empty((4, Cout), **f32)
        mean, invstd, scale, shift = vec[0], vec[1], vec[2], vec[3]
        _chk(lib.pdt_bn_finalize(_p(part), R, Cout, float(M), float(bna.eps), float(bna.momentum), _p(gamma),
                                 _p(beta), _p(mean), _p(invstd), _p(scale), _p(shift), _p(bna.rm), _p(bna.rv),
                                 _p(bna.nbt), st), "bn_finalize")
    else:
        invstd = torch.rsqrt(bna.rv.float() + bna.eps)
        mean = bna.rm.float().clone()
        scale = (gamma.float() * invstd).contiguous()
        shift = (beta.float() - mean * scale).contiguous()
    assert y.numel() == M * Cout
    if not apply:  # the consumer applies the BN affine (+ReLU) itself (stem max-pool)
        u = _Unit()
        u.x, u.w, u.gamma, u.beta, u.y = x, w, gamma, beta, y
        u.act, u.mask, u.bnb_pre, u.pend, u.res_unit = None, None, None, None, None
        u.mean, u.invstd, u.scale, u.shift = mean, invstd, scale, shift
        u.N, u.C, u.Cs, u.H, u.W, u.Cout, u.g, u.relu, u.has_res = N, C, Cs, H, W, Cout, g, relu, False
        return None, u
    res = None
    if residual is not None:
        res = _cl(residual)
        assert res.dtype == torch.bfloat16 and res.shape == y.shape, (res.shape, y.shape)
    out = torch.empty_like(y, memory_format=torch.channels_last)
    # residual + ReLU: the backward's ReLU mask cannot be recomputed from y alone; keep it
    # as one bit per element instead of re-reading the bf16 output (1/16 of the bytes)
    mask = torch.empty(M * Cout // 8, dtype=torch.uint8, device=x.device) if (relu and residual is not None) \
        else None
    if res_unit is not None:
        assert residual is res_unit.y and res_unit.Cout == Cout
    u = _Unit()
    u.pend = None
    if defer and relu:
        u.pend = (res, res_unit, out)
    elif res_unit is not None:
        _chk(lib.pdt_bn_apply_res_affine(_p(y), _p(res), _p(out), _p(scale), _p(shift), _p(res_unit.scale),
                                         _p(res_unit.shift), M, Cout, int(relu), _p(mask), st), "bn_apply_res_affine")
    else:
        _chk(lib.pdt_bn_apply(_p(y), _p(res), _p(out), _p(scale), _p(shift), M, Cout, int(relu), _p(mask), st),
             "bn_apply")
    u.x, u.w, u.gamma, u.beta, u.y = x, w, gamma, beta, y
    u.act = None
    u.mask = mask
    u.res_unit = res_unit  # the downsample unit whose raw output is this unit's residual (or None)
    u.bnb_pre = None
    u.mean, u.invstd, u.scale, u.shift = mean, invstd, scale, shift
    u.N, u.C, u.Cs, u.H, u.W, u.Cout, u.g, u.relu, u.has_res = N, C, Cs, H, W, Cout, g, relu, residual is not None
    return out, u


def _bn_bwd(dA, u: _Unit, want_dres: bool, mask=None, pre: _BnbPartials | None = None, coeffs_only=False):
    """BN(+res)(+ReLU) backward: returns (dy, dres, dgamma, dbeta). ``mask`` (a ReLU bit
    mask of another unit's output) gates dA first -- the downsample branch of a bottleneck
    sees the block's ReLU exactly as the main branch does. ``pre``: the reduction was
    already done by the epilogue of the GEMM that produced dA (no reduce pass).
    ``coeffs_only``: stop before the apply pass, return (dgamma, dbeta, k1, k2, k3)."""
    lib = _load()
    st = _s()
    dA = _cl(dA.to(torch.bfloat16))
    Cout = u.Cout
    M = u.N * u.g["Ho"] * u.g["Wo"]
    f32 = dict(dtype=torch.float32, device=dA.device)
    if mask is None:
        mask = u.mask
    relu = u.relu or mask is not None
    if pre is not None:
        assert pre.unit is u
        part, blocks = pre.part, pre.R
    else:
        blocks = lib.pdt_bn_stats_blocks(M, Cout)
        part = torch.empty(2 * blocks * Cout + lib.pdt_rows_reduce_workspace(blocks, Cout), **f32)
        _chk(lib.pdt_bn_bwd_reduce(_p(dA), _p(u.y), _p(u.act), _p(u.mean), _p(u.scale), _p(u.shift), _p(part), M,
                                   Cout, int(relu), blocks, _p(mask), st), "bn_bwd_reduce")
    vec = torch.empty((3, Cout), **f32)
    k1, k2, k3 = vec[0], vec[1], vec[2]
    dgamma, dbeta = _grad_buf(u.gamma, (Cout,)), _grad_buf(u.beta, (Cout,))
    _chk(lib.pdt_bn_bwd_finalize(_p(part), blocks, Cout, float(M), _p(u.gamma), _p(u.mean), _p(u.invstd),
                                 _p(dgamma), _p(dbeta), _p(k1), _p(k2), _p(k3), 0, st), "bn_bwd_finalize")
    if coeffs_only:
        return dgamma, dbeta, k1, k2, k3
    dy = torch.empty_like(u.y, memory_format=torch.channels_last)
    dres = torch.empty_like(u.y, memory_format=torch.channels_last) if want_dres else None
    _chk(lib.pdt_bn_bwd_apply(_p(dA), _p(u.y), _p(u.act), _p(u.scale), _p(u.shift), _p(k1), _p(k2), _p(k3),
                              _p(dy), _p(dres), M, Cout, int(relu), _p(mask), st), "bn_bwd_apply")
    return dy, dres, dgamma, dbeta


def _bn_bwd_pool(dout, idx, u: _Unit, k, s, p):
    """Stem BN+ReLU backward reading dA straight from the max-pool output gradient
    and argmax (csrc/bn_act.hip ``pdt_bn_bwd_*_pool``): the full-resolution dA of
    the ``maxpool_bwd`` + ``_bn_bwd`` composition is never materialised."""
    lib = _load()
    st = _s()
    N, C, H, W = u.N, u.Cout, u.g["Ho"], u.g["Wo"]
    Ho, Wo = dout.shape[2], dout.shape[3]
    assert dout.is_contiguous(memory_format=torch.channels_last) and dout.dtype == torch.bfloat16
    assert idx.numel() == N * Ho * Wo * C and u.y.shape == (N, C, H, W)
    assert u.relu and u.act is None and u.mask is None
    M = N * H * W
    f32 = dict(dtype=torch.float32, device=dout.device)
    # the gathered reduce is latency-bound (argmax byte -> gradient load chains): far
    # more blocks in flight than the streaming reduce's 512
    rp = 256 // (C // 8)
    blocks = max(1, min(int(os.environ.get("PDT_POOL_BN_BLOCKS", "4096")), (M + rp - 1) // rp))
    part = torch.empty(2 * blocks * C + lib.pdt_rows_reduce_workspace(blocks, C), **f32)
    _chk(lib.pdt_bn_bwd_reduce_pool(_p(dout), _p(idx), _p(u.y), _p(u.mean), _p(u.scale), _p(u.shift), _p(part),
                                    N, H, W, C, Ho, Wo, k, s, p, blocks, st), "bn_bwd_reduce_pool")
    vec = torch.empty((3, C), **f32)
    k1, k2, k3 = vec[0], vec[1], vec[2]
    dgamma, dbeta = _grad_buf(u.gamma, (C,)), _grad_buf(u.beta, (C,))
    _chk(lib.pdt_bn_bwd_finalize(_p(part), blocks, C, float(M), _p(u.gamma), _p(u.mean), _p(u.invstd),
                                 _p(dgamma), _p(dbeta), _p(k1), _p(k2), _p(k3), 0, st), "bn_bwd_finalize")
    dy = torch.empty_like(u.y, memory_format=torch.channels_last)
    _chk(lib.pdt_bn_bwd_apply_pool(_p(dout), _p(idx), _p(u.y), _p(u.scale), _p(u.shift), _p(k1), _p(k2), _p(k3),
                                   _p(dy), N, H, W, C, Ho, Wo, k, s, p, st), "bn_bwd_apply_pool")
    return dy, dgamma, dbeta


def _unit_dx(dy, u: _Unit, addend=None, addend_mask=None, bnb_unit=None, bnb_mask=None, bnb_unit2=None):
    """Data gradient of unit ``u``'s conv. With ``bnb_unit`` (the unit whose output
    this gradient flows into) returns ``(dx, _BnbPartials)``."""
    wd = u.w
    if u.Cs != u.C:  # stem: dgrad against the channel-padded weight, then drop the pad
        wd = torch.nn.functional.pad(u.w.detach().float(), (0, 0, 0, 0, 0, u.Cs - u.C))
        assert addend is None and bnb_unit is None
    dx = _conv_dgrad(dy, wd, u.N, u.H, u.W, u.Cs, u.Cout, u.g, addend=addend, addend_mask=addend_mask,
                     bnb_unit=bnb_unit, bnb_mask=bnb_mask, bnb_unit2=bnb_unit2)
    return dx[:, :u.C] if u.Cs != u.C else dx


# -----------------------------------------------------------------------------
# BatchNorm apply folded into a 1x1 GEMM's A staging (csrc/conv_nt_kernel.h AXArgs):
# the BN'd tensor is produced by the GEMM that consumes it (and written once for its
# other consumers) instead of by an element pass + a re-read. PDT_FUSE_BN_AX=0 disables.
# -----------------------------------------------------------------------------
AX_VARIANTS = (0, 1, 3, 5, 6, 8, 10, 13, 15, 16, 18, 20, 23, 25, 26, 28, 30, 31)  # csrc/conv_igemm_ax.hip


def _ax_enabled() -> bool:
    return os.environ.get("PDT_FUSE_BN_AX", "1") != "0"


def _conv1_fold_enabled() -> bool:
    """bn1's backward apply in conv1's data gradient (PDT_FUSE_BN_AX1=0 disables)."""
    return os.environ.get("PDT_FUSE_BN_AX1", "1") != "0"


def _ax_launch(lib, src, b, out, v, a, stats=None, bnb=None, ax=None):
    """One pdt_conv_nt_ax launch. ``bnb`` = (y, mean, scale, shift, mask, part, relu, row0, R) or None;
    ``ax`` = (mode, y2, c1, c2, c3, rsc, rsh, mask_in, mask_out, dst)."""
    bn = bnb if bnb is not None else (None, None, None, None, None, None, 0, 0, 0)
    mode, y2, c1, c2, c3, rsc, rsh, mki, mko, dst = ax
    return lib.pdt_conv_nt_ax(_p(src), _p(b), _p(out), _p(stats), a["Hs"], a["Ws"], a["Cs"], a["Nimg"], a["Hm"],
                              a["Wm"], a["Ncol"], a["K"], a["ldb"], a["ldo"], int(v), _p(bn[0]), _p(bn[1]),
                              _p(bn[2]), _p(bn[3]), _p(bn[4]), _p(bn[5]), int(bn[6]), int(bn[7]), int(bn[8]),
                              int(mode), _p(y2), _p(c1), _p(c2), _p(c3), _p(rsc), _p(rsh), _p(mki), _p(mko), _p(dst),
                              _s())


def _time_fn(fn):
    """Best of two 3-launch HIP-event trials after one warm call (``_time_variants``' protocol), ms."""
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    best = float("inf")
    for _ in range(2):
        ev0.record()
        for _ in range(3):
            fn()
        ev1.record()
        ev1.synchronize()
        best = min(best, ev0.elapsed_time(ev1))
    return best


AX_UNFUSED = -2  # tuned-table value: the element pass + the plain GEMM beat every AX tile here


def _ax2_launch(lib, src, b, out, v, a, stats=None, bnb=None, ax=None, addend=None, addend_mask=None):
    """``_ax_launch`` for any stride-1 geometry (``a`` as ``_fwd_nt_geom`` / ``_conv_dgrad`` build it);
    ``addend`` (+ ``addend_mask``): added in the fused BN-backward epilogue (modes 2 / 3)."""
    bn = bnb if bnb is not None else (None, None, None, None, None, None, 0, 0, 0)
    mode, y2, c1, c2, c3, rsc, rsh, mki, mko, dst = ax
    return lib.pdt_conv_nt_ax3(
        _p(src), _p(b), _p(out), _p(stats), _p(addend), _p(addend_mask), a["Hs"], a["Ws"], a["Cs"], a["Nimg"], a["Hm"], a["Wm"], a["Ncol"], a["K"],
        a["ldb"], a["sh"], a["sw"], a["oh0"], a["ow0"], a["dh"], a["dw"], a["nth"], a["ntw"], a["Ho"], a["Wo"],
        a["osh"], a["osw"], a["oph"], a["opw"], a["ldo"], int(v), _p(bn[0]), _p(bn[1]), _p(bn[2]), _p(bn[3]),
        _p(bn[4]), _p(bn[5]), int(bn[6]), int(bn[7]), int(bn[8]), int(mode), _p(y2), _p(c1), _p(c2), _p(c3), _p(rsc),
        _p(rsh), _p(mki), _p(mko), _p(dst), _s())


def _ax_select(key, run, run_ref=None):
    """Tile for an AX launch (tuned over the AX instantiations on first use when allowed);
    ``run(v)`` launches variant v (with the caller's scratch outputs) and returns its code.
    ``run_ref()``: the unfused alternative (element pass + the plain GEMM's tuned tile);
    when it is faster the key records ``AX_UNFUSED`` and the caller takes that path (the
    fold is a per-geometry tuning decision, not a blanket switch)."""
    table = _tuned()
    extra = os.environ.get("PDT_RETUNE_AX")  # targeted re-tune of shipped AX keys (as PDT_RETUNE_WITH)
    if key in table and not (extra and key not in _RETUNED and _tune_allowed()):
        return int(table[key])
    if not _tune_allowed():
        return AX_VARIANTS[3]  # 128x128, one LDS stage
    cand = set(AX_VARIANTS)
    if key in table:
        _RETUNED.add(key)
        cur = int(table[key])
        cand = _id_set(extra) | ({cur} if cur >= 0 else set())
    best = _time_variants(max(cand) + 1, run, cand)
    if best >= 0 and run_ref is not None and _time_fn(run_ref) < _time_fn(lambda: run(best)):
        best = AX_UNFUSED
    table[key] = best
    _save_tuned()
    return best


def _conv3_dgrad_bn_bwd(dout, u3, k1, k2, k3, dy3, u2, side=None):
    """Data gradient of a bottleneck's conv3 (1x1) with bn3's backward apply folded into its A
    staging: A = dy3 = k1*gate(dout) + k2*y3 + k3 (gate: u3's ReLU bit mask), written to ``dy3``
    for the weight gradient; bn2's backward partials in the epilogue (as ``_unit_dx(...,
    bnb_unit=u2)``). Returns (da2, _BnbPartials) or None when the geometry is not covered.
    ``side`` = (ud, b1, b2, b3, dyd): a downsample block's shortcut BN backward, otherwise
    applied together with bn3's by ``pdt_bn_bwd_apply_dual``; here it runs as its own pass and
    the tuner compares (fold + that pass) against (dual pass + plain data gradient)."""
    N, Cout, H, W = u3.y.shape
    Cin = u3.C
    if u3.g["KH"] != 1 or u3.g["sh"] != 1 or u3.Cs != Cin or Cout % 64 or u2.Cout != Cin or u3.mask is None:
        return None
    lib = _load()
    wt = _DGRAD_W.get(u3.w, Cout, 1, 1, Cin, 0, 0, 1, 1, 1)
    da2 = _empty_cl(N, Cin, H, W, torch.bfloat16, dout.device)
    a = dict(Hs=H, Ws=W, Cs=Cout, Nimg=N, Hm=H, Wm=W, Ncol=Cin, K=Cout, ldb=Cout, ldo=Cin)
    M = N * H * W
    assert u2.y.shape == da2.shape and u2.y.is_contiguous(memory_format=torch.channels_last)
    ax = (2, u3.y, k1, k2, k3, None, None, u3.mask, None, dy3)

    def bnb(part, R):
        return (u2.y, u2.mean, u2.scale, u2.shift, None, part, 1, 0, R)

    def run(v):
        R = lib.pdt_conv_nt_bnb_rows(M, Cin, Cout, v)
        part = torch.empty(2 * R * Cin, dtype=torch.float32, device=dout.device)
        return _ax_launch(lib, dout, wt, da2, v, a, bnb=bnb(part, R), ax=ax)

    def side_apply():
        ud, b1, b2, b3, dyd = side
        _chk(lib.pdt_bn_bwd_apply(_p(dout), _p(ud.y), None, None, None, _p(b1), _p(b2), _p(b3), _p(dyd), None, M,
                                  Cout, 1, _p(u3.mask), _s()), "bn_bwd_apply (shortcut)")

    def run_ref():
        if side is None:
            _chk(lib.pdt_bn_bwd_apply(_p(dout), _p(u3.y), None, None, None, _p(k1), _p(k2), _p(k3), _p(dy3), None,
                                      M, Cout, 1, _p(u3.mask), _s()), "bn_bwd_apply")
        else:
            ud, b1, b2, b3, dyd = side
            _chk(lib.pdt_bn_bwd_apply_dual(_p(dout), _p(u3.mask), _p(u3.y), _p(k1), _p(k2), _p(k3), _p(dy3),
                                           _p(ud.y), _p(b1), _p(b2), _p(b3), _p(dyd), M, Cout, _s()),
                 "bn_bwd_apply_dual")
        _unit_dx(dy3, u3, bnb_unit=u2)

    def run_tuned(v):
        rc = run(v)
        if rc == 0 and side is not None:
            side_apply()
        return rc

    key = ("axd:" if side is not None else "axb:") + ",".join(str(x) for x in (H, W, Cout, N, Cin))
    v = _ax_select(key, run_tuned, run_ref)
    if v < 0:
        return None
    R = lib.pdt_conv_nt_bnb_rows(M, Cin, Cout, v)
    part = torch.empty(2 * R * Cin + lib.pdt_rows_reduce_workspace(R, Cin), dtype=torch.float32, device=dout.device)
    rc = _ax_launch(lib, dout, wt, da2, v, a, bnb=bnb(part, R), ax=ax)
    if rc == NOT_APPLICABLE:
        return None
    _chk(rc, "conv_nt_ax (bn3 backward apply + conv3 dgrad)")
    if side is not None:
        side_apply()
    return da2, _BnbPartials(part, R, u2)


def _materialize(u: _Unit):
    """The deferred BN(+res)+ReLU element pass of unit ``u`` (see ``_unit_fwd(defer=True)``)."""
    _apply_pending(u)
    u.pend = None


def _apply_pending(u: _Unit):
    res, ru, out = u.pend
    lib = _load()
    M = u.y.numel() // u.Cout
    if ru is not None:
        _chk(lib.pdt_bn_apply_res_affine(_p(u.y), _p(res), _p(out), _p(u.scale), _p(u.shift), _p(ru.scale),
                                         _p(ru.shift), M, u.Cout, 1, _p(u.mask), _s()), "bn_apply_res_affine")
    else:
        _chk(lib.pdt_bn_apply(_p(u.y), _p(res), _p(out), _p(u.scale), _p(u.shift), M, u.Cout, 1, _p(u.mask), _s()),
             "bn_apply")


def _conv_fwd_ax(pu: _Unit, xbuf, wb, N, H, W, Cs, Cout, g, with_stats):
    """Forward stride-1 conv (1x1, or 3x3 'same') whose A operand is unit ``pu``'s deferred output
    relu(bn(pu.y) [+ res]), computed in the A staging (AX mode 1) and written to ``xbuf``
    (+ pu.mask) on the way. Returns ``_conv_forward``'s (y, M, part, R), or None when the
    geometry is not covered."""
    res, ru, _ = pu.pend
    Ho, Wo = g["Ho"], g["Wo"]
    M = N * Ho * Wo
    if g["sh"] != 1 or g["sw"] != 1 or Ho != H or Wo != W or Cs != pu.Cout or Cs % 64 or Cout % 8 or \
            N * H * W * Cs >= _AX_MAX_ELEMS or not pu.relu:
        return None
    lib = _load()
    y = _empty_cl(N, Cout, Ho, Wo, torch.bfloat16, xbuf.device)
    a = _fwd_nt_geom(N, H, W, Cs, Cout, g)
    K = a["K"]
    ax = (1, res, pu.scale, pu.shift, None, ru.scale if ru is not None else None,
          ru.shift if ru is not None else None, None, pu.mask, xbuf)

    def stats(v, tail):
        if not with_stats:
            return None, 0
        R = lib.pdt_conv_nt_stat_rows(M, Cout, K, v)
        ws = lib.pdt_rows_reduce_workspace(R, Cout) if tail else 0
        return torch.empty(2 * R * Cout + ws, dtype=torch.float32, device=xbuf.device), R

    def run(v):
        return _ax2_launch(lib, pu.y, wb, y, v, a, stats=stats(v, False)[0], ax=ax)

    def run_ref():
        _apply_pending(pu)
        _conv_forward(xbuf, wb, N, H, W, Cs, Cout, g, with_stats=with_stats)

    key = "axf:" + ",".join(str(x) for x in (H, W, Cs, N, Cout, int(res is not None), int(ru is not None),
                                              int(with_stats)))
    if g["KH"] != 1 or g["KW"] != 1:
        key += f",k{g['KH']}x{g['KW']}p{g['ph']}"
    v = _ax_select(key, run, run_ref)
    if v < 0:
        return None
    part, R = stats(v, True)
    rc = _ax2_launch(lib, pu.y, wb, y, v, a, stats=part, ax=ax)
    if rc == NOT_APPLICABLE:
        return None
    _chk(rc, "conv_nt_ax (deferred BN apply + conv)")
    return y, M, part, R


def _conv2_dgrad_bn_bwd(da2, u2, k1, k2, k3, dy2, u1, bnb_mask=None, addend=None, addend_mask=None):
    """Data gradient of a bottleneck's stride-1 conv2 (3x3) with bn2's backward apply folded into
    its A staging (AX mode 3: dy2 = k1*gate(da2) + k2*y2 + k3, the ReLU gate recomputed from y2
    as ``pdt_bn_bwd_apply`` does), dy2 written once (centre tap) for the weight gradient; bn1's
    backward partials in the epilogue. Returns (da1, _BnbPartials) or None (not covered / the
    element pass + plain data gradient tuned faster).
    The same fold serves conv1's data gradient (``u2`` = the block's conv1 unit, ``u1`` = the
    previous block's conv3 unit, ``bnb_mask`` = its ReLU bit mask): there the epilogue also adds
    the shortcut gradient ``addend`` (gated by ``addend_mask``), as ``_unit_dx`` does."""
    g = u2.g
    N, Cout, Ho, Wo = u2.y.shape
    Cin = u2.C
    if g["sh"] != 1 or g["sw"] != 1 or Ho != u2.H or Wo != u2.W or u2.Cs != Cin or Cout % 64 or u1.Cout != Cin or \
            u2.mask is not None or not u2.relu or N * Ho * Wo * Cout >= _AX_MAX_ELEMS:
        return None
    KH, KW, ph, pw = g["KH"], g["KW"], g["ph"], g["pw"]
    lib = _load()
    wt = _DGRAD_W.get(u2.w, Cout, KH, KW, Cin, 0, 0, 1, KH, KW)
    da1 = _empty_cl(N, Cin, u2.H, u2.W, torch.bfloat16, da2.device)
    a = dict(Hs=Ho, Ws=Wo, Cs=Cout, Nimg=N, Hm=u2.H, Wm=u2.W, Ncol=Cin, K=KH * KW * Cout, ldb=KH * KW * Cout, sh=1,
             sw=1, oh0=ph, ow0=pw, dh=-1, dw=-1, nth=KH, ntw=KW, Ho=u2.H, Wo=u2.W, osh=1, osw=1, oph=0, opw=0,
             ldo=Cin)
    M = N * u2.H * u2.W
    ax = (3, u2.y, k1, k2, k3, u2.scale, u2.shift, None, None, dy2)
    if addend is not None:
        _check_addend(addend, da1, addend_mask, Cin)
    if bnb_mask is not None:
        assert bnb_mask.dtype == torch.uint8 and bnb_mask.numel() * 8 == da1.numel()

    def bnb(part, R):
        return (u1.y, u1.mean, u1.scale, u1.shift, bnb_mask, part, 1, 0, R)

    def run(v):
        R = lib.pdt_conv_nt_bnb_rows(M, Cin, a["K"], v)
        part = torch.empty(2 * R * Cin, dtype=torch.float32, device=da2.device)
        return _ax2_launch(lib, da2, wt, da1, v, a, bnb=bnb(part, R), ax=ax, addend=addend, addend_mask=addend_mask)

    def run_ref():
        _chk(lib.pdt_bn_bwd_apply(_p(da2), _p(u2.y), None, _p(u2.scale), _p(u2.shift), _p(k1), _p(k2), _p(k3),
                                  _p(dy2), None, N * Ho * Wo, Cout, 1, None, _s()), "bn_bwd_apply")
        _unit_dx(dy2, u2, addend=addend, addend_mask=addend_mask, bnb_unit=u1, bnb_mask=bnb_mask)

    key = "ax3:" + ",".join(str(x) for x in (Ho, Wo, Cout, N, Cin, KH, KW, ph))
    if addend is not None or bnb_mask is not None:
        key += f",a{int(addend is not None)}{int(addend_mask is not None)}m{int(bnb_mask is not None)}"
    v = _ax_select(key, run, run_ref)
    if v < 0:
        return None
    R = lib.pdt_conv_nt_bnb_rows(M, Cin, a["K"], v)
    part = torch.empty(2 * R * Cin + lib.pdt_rows_reduce_workspace(R, Cin), dtype=torch.float32, device=da2.device)
    rc = _ax2_launch(lib, da2, wt, da1, v, a, bnb=bnb(part, R), ax=ax, addend=addend, addend_mask=addend_mask)
    if rc == NOT_APPLICABLE:
        return None
    _chk(rc, "conv_nt_ax (BN backward apply + conv dgrad)")
    return da1, _BnbPartials(part, R, u1)


def _unit_dw(dy, u: _Unit):
    w = u.w
    KH, KW = u.g["KH"], u.g["KW"]
    if u.Cs == u.C and w.is_contiguous(memory_format=torch.channels_last):
        dw = _grad_buf(w, tuple(w.shape), torch.channels_last)
        _conv_wgrad(dy, u.x, u.N, u.H, u.W, u.Cs, u.Cout, u.g, dw)
    else:
        tmp = torch.empty((u.Cout, u.Cs, KH, KW), dtype=torch.float32, device=dy.device,
                          memory_format=torch.channels_last)
        _conv_wgrad(dy, u.x, u.N, u.H, u.W, u.Cs, u.Cout, u.g, tmp)
        dw = _grad_buf(w, tuple(w.shape), torch.channels_last).copy_(tmp[:, :u.C]) if u.Cs != u.C else tmp
    return dw.to(w.dtype) if dw.dtype != w.dtype else dw


class _ConvBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gamma, beta, residual, conv, relu, bna):
        out, u = _unit_fwd(x, w, gamma, beta, residual, conv, relu, bna)
        ctx.u = u
        ctx.save_for_backward(u.x, u.y, u.mask)  # version-checked activations
        return out

    @staticmethod
    def backward(ctx, dA):
        u = ctx.u
        dy, dres, dgamma, dbeta = _bn_bwd(dA, u, u.has_res)
        dx = _unit_dx(dy, u) if ctx.needs_input_grad[0] else None
        dw = _unit_dw(dy, u) if ctx.needs_input_grad[1] else None
        del ctx.u
        return (dx, dw, dgamma if ctx.needs_input_grad[2] else None, dbeta if ctx.needs_input_grad[3] else None,
                dres, None, None, None)


def conv_bn_act(x, conv: nn.Conv2d, bn: nn.BatchNorm2d, residual=None, relu=True):
    if not supports_conv(x, conv) or (residual is not None and residual.dtype != torch.bfloat16):
        fallback("conv_bn_act", f"conv {tuple(conv.kernel_size)}/{tuple(conv.stride)} groups={conv.groups} "
                                f"bias={conv.bias is not None} on {tuple(x.shape)} {x.dtype}")
        from .fused import _torch_conv_bn_act
        return _torch_conv_bn_act(x, conv, bn, residual, relu)
    return _ConvBNAct.apply(x, conv.weight, bn.weight, bn.bias, residual, conv, relu, _BNArgs(bn))


# =============================================================================
# fused ResNet bottleneck: conv1-bn1-relu -> conv2-bn2-relu -> conv3-bn3 (+ identity
# or downsample conv-bn) -> relu, with a hand-scheduled backward: the block-input
# gradient is produced by ONE data-gradient GEMM whose epilogue adds the
# identity / downsample branch gradient (no separate add pass).
# =============================================================================
# Cross-block fusion of the BatchNorm-backward reduction. Block k's output is
# block k+1's input; block k+1's backward produces that gradient with ONE dgrad
# GEMM (+ shortcut addend), so its epilogue also computes block k's bn3
# backward partials (gated by block k's ReLU bit mask). Forward records which
# unit produced each block output; backward leaves the partials on that unit,
# tagged with the gradient tensor's storage and version -- block k's backward
# uses them only if the gradient it receives is exactly that tensor.
_PRODUCERS: dict = {}


def _note_producer(out, u):
    if len(_PRODUCERS) > 64:
        for k in [k for k, e in _PRODUCERS.items() if e[0]() is None]:
            del _PRODUCERS[k]
    _PRODUCERS[out.data_ptr()] = (weakref.ref(u), tuple(out.shape), out.stride(), out._version)


def _producer_of(x):
    e = _PRODUCERS.get(x.data_ptr())
    if e is None:
        return None
    u = e[0]()
    if u is None or e[1] != tuple(x.shape) or e[2] != x.stride() or e[3] != x._version:
        return None
    return u


def _take_bnb(u, grad):
    """Partials a later block's epilogue left for unit ``u``, if ``grad`` is that output."""
    st, u.bnb_pre = u.bnb_pre, None
    if st is None or st[0] != grad.data_ptr() or st[1] != grad._version or st[2] != tuple(grad.shape):
        return None
    return st[3]


# (Weight gradients on a side HIP stream beside the data-gradient chain were an opt-in switch
# through round 5: +0.4 % / -0.3 % at bs 512 / 256, and at bs 2048 on the round-6 tree 1 163 vs
# 14 573 img/s -- the stream-recorded blocks of the 85-GiB step kept the caching allocator from
# reusing memory (profiles/bench_runs_round6.jsonl, call q04). Removed: one stream.)


class _Bottleneck(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blk, has_ds, xpend, defer, holder, *params):
        # xpend: the previous block's unit whose output x is still unwritten (its bn3 apply is
        # computed in conv1's A staging, which writes x); conv1 therefore runs first
        fold = _ax_enabled()
        # bn1's apply+ReLU inside conv2's A staging when conv2 is stride 1 (a1 written once, at
        # the centre tap, for conv2's weight gradient); otherwise materialised before conv2
        a1, u1 = _unit_fwd(x, blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, None, blk.conv1, True,
                           _BNArgs(blk.bn1), src_pend=xpend, defer=fold)
        if has_ds:  # raw downsample conv output; its BN affine is applied inside bn3's apply
            _, ud = _unit_fwd(x, blk.downsample[0].weight, blk.downsample[1].weight, blk.downsample[1].bias, None,
                              blk.downsample[0], False, _BNArgs(blk.downsample[1]), apply=False)
            idn = ud.y
        else:
            idn, ud = _cl(x.to(torch.bfloat16)), None
        # bn2's apply+ReLU inside conv3's A staging (a2 written once, for conv3's weight gradient)
        a2, u2 = _unit_fwd(a1, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias, None, blk.conv2, True,
                           _BNArgs(blk.bn2), src_pend=u1, defer=fold)
        out, u3 = _unit_fwd(a2, blk.conv3.weight, blk.bn3.weight, blk.bn3.bias, idn, blk.conv3, True,
                            _BNArgs(blk.bn3), res_unit=ud, src_pend=u2, defer=defer and fold)
        if holder is not None:
            holder[0] = u3 if u3.pend is not None else None
        ctx.units = (u1, u2, u3, ud)
        ctx.has_ds = has_ds
        prev = _producer_of(x) if _bnb_enabled() else None
        ctx.prev = weakref.ref(prev) if prev is not None else None
        ctx.save_for_backward(u1.x, u1.y, u2.y, u3.y, u3.mask)
        _note_producer(out, u3)
        return out

    @staticmethod
    def backward(ctx, dout):
        u1, u2, u3, ud = ctx.units
        need = ctx.needs_input_grad
        dout = _cl(dout.to(torch.bfloat16))
        # bn3's backward partials from the next block's data-gradient epilogue (and, in a
        # downsample block, the shortcut BN's from the same epilogue: same gated gradient)
        pre3 = _take_bnb(u3, dout)
        pre_d = pre3.second if (pre3 is not None and pre3.second is not None and pre3.second.unit is ud) else None
        dual = ctx.has_ds and u3.mask is not None and os.environ.get("PDT_BN_DUAL_APPLY", "1") == "1"
        if dual:
            # both BN backwards fed by dout (bn3 and the shortcut's BN): coefficients first, then
            # ONE apply pass that reads dout and the ReLU mask once and writes both gradients
            dg3, db3, a1, a2, a3 = _bn_bwd(dout, u3, False, pre=pre3, coeffs_only=True)
            dgd, dbd, b1, b2, b3 = _bn_bwd(dout, ud, False, mask=u3.mask, pre=pre_d, coeffs_only=True)
            dy3 = torch.empty_like(u3.y, memory_format=torch.channels_last)
            dyd = torch.empty_like(ud.y, memory_format=torch.channels_last)
            fused3 = None
            if _bnb_enabled() and _ax_enabled():  # bn3's half in conv3's A staging (when it wins)
                fused3 = _conv3_dgrad_bn_bwd(dout, u3, a1, a2, a3, dy3, u2, side=(ud, b1, b2, b3, dyd))
            if fused3 is None:
                M3 = u3.N * u3.g["Ho"] * u3.g["Wo"]
                _chk(_load().pdt_bn_bwd_apply_dual(_p(dout), _p(u3.mask), _p(u3.y), _p(a1), _p(a2), _p(a3),
                                                   _p(dy3), _p(ud.y), _p(b1), _p(b2), _p(b3), _p(dyd), M3, u3.Cout,
                                                   _s()), "bn_bwd_apply_dual")
        else:
            fused3 = None
        fuse = _bnb_enabled()
        if not dual and fuse and _ax_enabled() and u3.mask is not None:
            # bn3's backward apply inside conv3's data-gradient A staging (dy3 written once, for
            # the weight gradient): no separate element pass, no re-read of dy3 by the dgrad
            dg3, db3, k1, k2, k3 = _bn_bwd(dout, u3, False, pre=pre3, coeffs_only=True)
            dy3 = torch.empty_like(u3.y, memory_format=torch.channels_last)
            fused3 = _conv3_dgrad_bn_bwd(dout, u3, k1, k2, k3, dy3, u2)
            if fused3 is None:  # not covered: the element pass
                _chk(_load().pdt_bn_bwd_apply(_p(dout), _p(u3.y), None, _p(u3.scale), _p(u3.shift), _p(k1), _p(k2),
                                              _p(k3), _p(dy3), None, u3.y.numel() // u3.Cout, u3.Cout, 1,
                                              _p(u3.mask), _s()), "bn_bwd_apply")
        elif not dual:
            dy3, _, dg3, db3 = _bn_bwd(dout, u3, False, pre=pre3)
        if fused3 is not None:
            da2, pre2 = fused3
        elif fuse:  # bn2 / bn1 backward reductions in the epilogues of the conv3 / conv2 dgrads
            da2, pre2 = _unit_dx(dy3, u3, bnb_unit=u2)
        else:
            da2, pre2 = _unit_dx(dy3, u3), None
        dw3 = _unit_dw(dy3, u3)
        fused2 = None
        if fuse and _ax_enabled():
            # bn2's backward apply inside conv2's data gradient (stride-1 conv2; tuned per shape)
            dg2, db2, c1, c2, c3 = _bn_bwd(da2, u2, False, pre=pre2, coeffs_only=True)
            dy2 = torch.empty_like(u2.y, memory_format=torch.channels_last)
            fused2 = _conv2_dgrad_bn_bwd(da2, u2, c1, c2, c3, dy2, u1)
            if fused2 is None:
                _chk(_load().pdt_bn_bwd_apply(_p(da2), _p(u2.y), None, _p(u2.scale), _p(u2.shift), _p(c1), _p(c2),
                                              _p(c3), _p(dy2), None, u2.y.numel() // u2.Cout, u2.Cout, 1, None,
                                              _s()), "bn_bwd_apply")
        else:
            dy2, _, dg2, db2 = _bn_bwd(da2, u2, False, pre=pre2)
        if fused2 is not None:
            da1, pre1 = fused2
        elif fuse:
            da1, pre1 = _unit_dx(dy2, u2, bnb_unit=u1)
        else:
            da1, pre1 = _unit_dx(dy2, u2), None
        dw2 = _unit_dw(dy2, u2)
        prev = ctx.prev() if ctx.prev is not None else None
        fold1 = fuse and _ax_enabled() and need[0] and prev is not None and prev.mask is not None and \
            prev.Cout == u1.C and u1.Cs == u1.C and _conv1_fold_enabled()
        if fold1:  # bn1's backward apply inside conv1's data gradient (below)
            dg1, db1, e1, e2, e3 = _bn_bwd(da1, u1, False, pre=pre1, coeffs_only=True)
            dy1 = torch.empty_like(u1.y, memory_format=torch.channels_last)
        else:
            dy1, _, dg1, db1 = _bn_bwd(da1, u1, False, pre=pre1)
        grads_ds = ()
        # shortcut gradient = dout * relu_mask(out): never materialised -- the downsample
        # BN backward gates dout with the mask itself, and an identity shortcut is added
        # (masked) by the epilogue of the block-input dgrad GEMM
        addend_mask = None
        if ctx.has_ds:
            if not dual:
                dyd, _, dgd, dbd = _bn_bwd(dout, ud, False, mask=u3.mask, pre=pre_d)
            addend = _unit_dx(dyd, ud) if need[0] else None
            dwd = _unit_dw(dyd, ud)
            grads_ds = (dwd, dgd, dbd)
        else:
            addend, addend_mask = dout, u3.mask
        dx = None
        if fold1:
            r1 = _conv2_dgrad_bn_bwd(da1, u1, e1, e2, e3, dy1, prev, bnb_mask=prev.mask, addend=addend,
                                     addend_mask=addend_mask)
            if r1 is not None:
                dx, pre = r1
                prev.bnb_pre = (dx.data_ptr(), dx._version, tuple(dx.shape), pre)
            else:  # not covered / tuned slower: the element pass, then the plain data gradient below
                _chk(_load().pdt_bn_bwd_apply(_p(da1), _p(u1.y), None, _p(u1.scale), _p(u1.shift), _p(e1), _p(e2),
                                              _p(e3), _p(dy1), None, u1.y.numel() // u1.Cout, u1.Cout, 1, None,
                                              _s()), "bn_bwd_apply")
        if dx is not None:
            pass
        elif need[0] and prev is not None and prev.mask is not None and prev.Cout == u1.C and u1.Cs == u1.C:
            # the previous block's bn3 backward partials from this epilogue (and its shortcut
            # BN's, when it is a downsample block)
            dx, pre = _unit_dx(dy1, u1, addend=addend, addend_mask=addend_mask, bnb_unit=prev, bnb_mask=prev.mask,
                               bnb_unit2=prev.res_unit if _bnb2_enabled() else None)
            prev.bnb_pre = (dx.data_ptr(), dx._version, tuple(dx.shape), pre)
        elif need[0]:
            dx = _unit_dx(dy1, u1, addend=addend, addend_mask=addend_mask)
        dw1 = _unit_dw(dy1, u1)
        del ctx.units
        return (dx, None, None, None, None, None, dw1, dg1, db1, dw2, dg2, db2, dw3, dg3, db3) + grads_ds


def _bottleneck_params(blk):
    params = [blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias,
              blk.conv3.weight, blk.bn3.weight, blk.bn3.bias]
    if blk.downsample is not None:
        params += [blk.downsample[0].weight, blk.downsample[1].weight, blk.downsample[1].bias]
    return params


def _bottleneck_ok(x, blk):
    convs = [blk.conv1, blk.conv2, blk.conv3] + ([blk.downsample[0]] if blk.downsample is not None else [])
    return x.dtype == torch.bfloat16 and all(supports_conv(x, c) for c in convs) and x.shape[1] % 8 == 0


def bottleneck(x, blk):
    if not _bottleneck_ok(x, blk):
        fallback("bottleneck", f"input {tuple(x.shape)} {x.dtype} (needs bf16, channels % 8 == 0, "
                               "plain convs)")
        return None
    return _Bottleneck.apply(x, blk, blk.downsample is not None, None, False, None, *_bottleneck_params(blk))


def bottleneck_chain(x, blocks):
    """A sequence of bottleneck blocks, one autograd node per block (DDP's per-parameter
    gradient hooks keep firing block by block), with each block's final BN(+residual)+ReLU
    element pass deferred into the NEXT block's conv1: that 1x1 GEMM computes the block
    output in its A staging and writes it (+ ReLU bit mask) once for the shortcut and the
    backward -- one full read of every block output per step saved. The deferred output is
    only ever read by the next block of this chain, which runs immediately after; the last
    block's output is materialised normally. Returns ``(y, n)``: ``blocks[:n]`` ran here
    (n < len(blocks) when block n is not covered -- the caller runs the rest)."""
    blocks = list(blocks)
    pend = None
    for i, blk in enumerate(blocks):
        if not _bottleneck_ok(x, blk):
            assert pend is None
            return x, i
        holder = [None]
        defer = i + 1 < len(blocks)
        x = _Bottleneck.apply(x, blk, blk.downsample is not None, pend, defer, holder, *_bottleneck_params(blk))
        pend = holder[0]
        if pend is not None and not _bottleneck_ok(x, blocks[i + 1]):
            _materialize(pend)
            pend = None
    assert pend is None
    return x, len(blocks)


# =============================================================================
# pooling
# =============================================================================
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        x = _cl(x)
        N, C, H, W = x.shape
        Ho = (H + 2 * p - k) // s + 1
        Wo = (W + 2 * p - k) // s + 1
        y = _empty_cl(N, C, Ho, Wo, torch.bfloat16, x.device)
        idx = torch.empty(N * Ho * Wo * C, dtype=torch.uint8, device=x.device)
        _chk(_load().pdt_maxpool_fwd(_p(x), _p(y), _p(idx), N, H, W, C, Ho, Wo, k, s, p, _s()), "maxpool_fwd")
        ctx.save_for_backward(idx)
        ctx.meta = (N, C, H, W, Ho, Wo, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W, Ho, Wo, k, s, p = ctx.meta
        dy = _cl(dy.to(torch.bfloat16))
        dx = _empty_cl(N, C, H, W, torch.bfloat16, dy.device)
        _chk(_load().pdt_maxpool_bwd(_p(dy), _p(idx), _p(dx), N, H, W, C, Ho, Wo, k, s, p, _s()), "maxpool_bwd")
        return dx, None, None, None


# -----------------------------------------------------------------------------
# Space-to-depth stem. The 7x7 stride-2 conv over 3 channels, run directly, pads
# every pixel to 8 channels (5/8 of the GEMM K is zeros) and gathers 49 taps of
# 16 B. Over NHWC storage padded to 4 channels, one 16-B chunk is instead TWO
# horizontally adjacent pixels: the conv becomes 8 (kh) x 4 (kw pairs) taps of
# 8 "channels" (b, c), K = 256 instead of 392, with the stride-2 column walk
# folded into the tap offset (ow0 = -4, dw = 2: every pair starts on an even
# pixel, so it is 16-B aligned and either wholly inside or wholly outside the
# image). The kernels take the pixel stride separately (pix = 4, Cs = 8).
#   W'[co, (kh*4 + t)*8 + b*4 + c] = W[co, c, kh, 2t + b - 1]  (0 outside 7x7 / c >= C)
# -----------------------------------------------------------------------------
_S2D_W: dict = {}


def _s2d_ok(x, conv: nn.Conv2d) -> bool:
    return (tuple(conv.kernel_size) == (7, 7) and tuple(conv.stride) == (2, 2) and tuple(conv.padding) == (3, 3)
            and conv.in_channels <= 4 and x.shape[1] == conv.in_channels and x.shape[2] % 2 == 0
            and x.shape[3] % 2 == 0 and os.environ.get("PDT_STEM_S2D", "1") != "0")


def _s2d_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, 256] bf16 space-to-depth stem weight (cached per parameter version)."""
    ent = _S2D_W.get(id(w))
    if ent is not None and ent[1] == w._version and ent[2] == w.data_ptr() and _same_tensor(ent[3], w):
        return ent[0]
    Cout, C = w.shape[0], w.shape[1]
    wp = torch.nn.functional.pad(w.detach().float(), (1, 0, 0, 1, 0, 4 - C))  # [Cout, 4, 8(kh), 8(kw+1)]
    out = wp.view(Cout, 4, 8, 4, 2).permute(0, 2, 3, 4, 1).reshape(Cout, 256).to(torch.bfloat16).contiguous()
    _S2D_W[id(w)] = (out, w._version, w.data_ptr(), _weak(w))
    return out


def _s2d_unfold_grad(dw256: torch.Tensor, C: int) -> torch.Tensor:
    """[Cout, 256] fp32 space-to-depth weight gradient -> [Cout, C, 7, 7]."""
    Cout = dw256.shape[0]
    g = dw256.view(Cout, 8, 4, 2, 4).permute(0, 4, 1, 2, 3).reshape(Cout, 4, 8, 8)
    return g[:, :C, :7, 1:8]


def _s2d_geom(N, H, W, Cout):
    Ho, Wo = H // 2, W // 2
    return dict(Hs=H, Ws=W, Cs=8, Nimg=N, Hm=Ho, Wm=Wo, Ncol=Cout, K=256, ldb=256, sh=2, sw=2, oh0=-3, ow0=-4,
                dh=1, dw=2, nth=8, ntw=4, Ho=Ho, Wo=Wo, osh=1, osw=1, oph=0, opw=0, ldo=Cout, pix=4)


def _stem_halo_choice(x4, wb, y, N, H, W, Cout, a, v) -> bool:
    """Halo-patch stem kernel (csrc/stem.hip) or the generic space-to-depth GEMM (tile ``v``):
    a tuned per-geometry choice (both with their BN statistics epilogue); ``PDT_STEM_HALO=0``
    forces the generic GEMM."""
    lib = _load()
    if os.environ.get("PDT_STEM_HALO", "1") == "0" or lib.pdt_stem_fwd_rows(N, H, W, Cout) < 0:
        return False
    key = f"stem1:{N},{H},{W},{Cout}"
    table = _tuned()
    if key in table:
        return int(table[key]) == 1
    if not _tune_allowed():
        return True
    f32 = dict(dtype=torch.float32, device=x4.device)
    Rh = lib.pdt_stem_fwd_rows(N, H, W, Cout)
    ph = torch.empty(2 * Rh * Cout, **f32)
    Rg = conv_stat_rows(N * H * W // 4, Cout, a["K"], v)
    pg = torch.empty(2 * Rg * Cout, **f32)

    def launch(k):
        if k == 1:
            return lib.pdt_stem_fwd(_p(x4), _p(wb), _p(y), _p(ph), N, H, W, Cout, _s())
        return lib.pdt_conv_nt(*_nt_args(x4, wb, y, pg, None, a, 0, v))
    table[key] = _time_variants(2, launch)
    _save_tuned()
    return int(table[key]) == 1


def _unit_fwd_s2d(x, w, gamma, beta, bna: _BNArgs):
    """Stem conv (space-to-depth GEMM) + BN statistics/finalize; no apply."""
    lib = _load()
    st = _s()
    N, C, H, W = x.shape
    x4 = nhwc_padded_view(x, 4)
    if x4 is None:
        x4 = _cl(torch.nn.functional.pad(_cl(x.to(torch.bfloat16)).permute(0, 2, 3, 1), (0, 4 - C))
                 .permute(0, 3, 1, 2))
    Cout = w.shape[0]
    a = _s2d_geom(N, H, W, Cout)
    Ho, Wo = a["Ho"], a["Wo"]
    M = N * Ho * Wo
    wb = _s2d_weight(w)
    y = _empty_cl(N, Cout, Ho, Wo, torch.bfloat16, x.device)
    f32 = dict(dtype=torch.float32, device=x.device)
    v = select_nt_variant(x4, wb, y, with_stats=bna.training, **a)
    halo = _stem_halo_choice(x4, wb, y, N, H, W, Cout, a, v) if bna.training else False
    if halo:  # the halo-patch stem kernel (csrc/stem.hip), statistics in its epilogue
        R = lib.pdt_stem_fwd_rows(N, H, W, Cout)
        part = torch.empty(2 * R * Cout + lib.pdt_rows_reduce_workspace(R, Cout), **f32)
        _chk(lib.pdt_stem_fwd(_p(x4), _p(wb), _p(y), _p(part), N, H, W, Cout, st), "stem_fwd")
    elif bna.training:
        R = conv_stat_rows(M, Cout, a["K"], v)
        part = torch.empty(2 * R * Cout + lib.pdt_rows_reduce_workspace(R, Cout), **f32)
        conv_nt(x4, wb, y, stats=part, variant=v, **a)
    if bna.training:
        vec = torch.empty((4, Cout), **f32)
        mean, invstd, scale, shift = vec[0], vec[1], vec[2], vec[3]
        _chk(lib.pdt_bn_finalize(_p(part), R, Cout, float(M), float(bna.eps), float(bna.momentum), _p(gamma),
                                 _p(beta), _p(mean), _p(invstd), _p(scale), _p(shift), _p(bna.rm), _p(bna.rv),
                                 _p(bna.nbt), st), "bn_finalize")
    else:
        conv_nt(x4, wb, y, variant=v, **a)
        invstd = torch.rsqrt(bna.rv.float() + bna.eps)
        mean = bna.rm.float().clone()
        scale = (gamma.float() * invstd).contiguous()
        shift = (beta.float() - mean * scale).contiguous()
    u = _Unit()
    u.x, u.w, u.gamma, u.beta, u.y = x4, w, gamma, beta, y
    u.act, u.mask, u.bnb_pre = None, None, None
    u.mean, u.invstd, u.scale, u.shift = mean, invstd, scale, shift
    g = dict(KH=7, KW=7, sh=2, sw=2, ph=3, pw=3, Ho=Ho, Wo=Wo, s2d=True)
    u.N, u.C, u.Cs, u.H, u.W, u.Cout, u.g, u.relu, u.has_res = N, C, 8, H, W, Cout, g, True, False
    return u


def _stem_wgrad_halo(u: _Unit, dA, coef, dw256, generic) -> bool:
    """The halo-patch stem weight gradient (csrc/stem.hip, the BN backward apply in its dY
    staging) into ``dw256``: variant 0 (register prefetch, 4-row bands) or 1 (all operands by
    LDS-DMA, double-buffered 2-row bands), a tuned per-geometry choice against each other and
    ``generic()`` (the generic weight-gradient path, itself tuned; key stem2w, value -1 =
    generic; ``PDT_STEM_HALO=0`` forces generic). False: not taken here (the caller runs
    ``generic``)."""
    lib = _load()
    N, H, W, Cout = u.N, u.H, u.W, u.Cout
    if os.environ.get("PDT_STEM_HALO", "1") == "0" or u.x.shape[1] != 4 or \
            lib.pdt_stem_wgrad_splits_v(N, H, W, Cout, 0) < 0:
        return False
    ws = {}

    def run_halo(v):
        splits = lib.pdt_stem_wgrad_splits_v(N, H, W, Cout, v)
        if splits < 0:
            return NOT_APPLICABLE
        if v not in ws:
            ws[v] = torch.empty(lib.pdt_wgrad_workspace(splits, Cout, 256), dtype=torch.float32, device=dA.device)
        rc = lib.pdt_stem_wgrad_v(_p(u.x), _p(dA), _p(u.y), _p(coef), _p(ws[v]), N, H, W, Cout, v, _s())
        if rc == 0:
            rc = lib.pdt_wgrad_reduce(_p(ws[v]), _p(dw256), None, None, splits, Cout, 256, 1.0, 0, _s())
        return rc

    key = f"stem2w:{N},{H},{W},{Cout}"
    table = _tuned()
    if key in table:
        choice = int(table[key])
    elif not _tune_allowed():
        choice = 1
    else:
        choice = _time_variants(2, run_halo)
        generic()  # settles the generic path's own tuning before it is timed
        if choice < 0 or _time_fn(generic) < _time_fn(lambda: run_halo(choice)):
            choice = -1
        table[key] = choice
        _save_tuned()
    if choice < 0:
        return False
    _chk(run_halo(choice), "stem_wgrad")
    return True


def _unit_dw_s2d(dy, u: _Unit, bn_dA=None):
    """Stem weight gradient (space-to-depth GEMM). ``bn_dA`` = (dA, k1, k2, k3): ``dy`` is
    not given (None) and the stem BN's backward apply is formed inside the weight
    gradient's dY staging when the tuner finds that faster than the element pass."""
    a = _s2d_geom(u.N, u.H, u.W, u.Cout)
    dw256 = torch.empty((u.Cout, 256), dtype=torch.float32, device=u.y.device)
    g = dict(M=u.N * a["Ho"] * a["Wo"], Mo=u.Cout, No=256, ldy=u.Cout, Hs=u.H, Ws=u.W, C=8, Hm=a["Ho"], Wm=a["Wo"],
             sh=2, sw=2, oh0=-3, ow0=-4, dh=1, dw=2, ntw=4, pix=4)
    if bn_dA is not None:
        dA, k1, k2, k3 = bn_dA
        coef = torch.stack([k1, k2, k3, u.scale, u.shift]).contiguous()
        lib = _load()
        M = u.y.numel() // u.Cout

        def apply_pass():
            dy = torch.empty_like(u.y, memory_format=torch.channels_last)
            _chk(lib.pdt_bn_bwd_apply(_p(dA), _p(u.y), None, _p(u.scale), _p(u.shift), _p(k1), _p(k2), _p(k3),
                                      _p(dy), None, M, u.Cout, 1, None, _s()), "bn_bwd_apply")
            return dy

        def run_ref():
            conv_wgrad(apply_pass(), u.x, dw256, **g)

        def generic():
            if not conv_wgrad_bn(dA, u.x, dw256, u.y, coef, run_ref, **g):
                conv_wgrad(apply_pass(), u.x, dw256, **g)

        if not _stem_wgrad_halo(u, dA, coef, dw256, generic):
            generic()
    else:
        conv_wgrad(dy, u.x, dw256, **g)
    dw = _grad_buf(u.w, tuple(u.w.shape), torch.channels_last).copy_(_s2d_unfold_grad(dw256, u.C))
    return dw.to(u.w.dtype) if dw.dtype != u.w.dtype else dw


def _pool_bwd_bnred(dout, idx, dA, u: _Unit, k, s, p):
    """Stem max-pool backward fused with the stem BN backward reduction
    (``pdt_maxpool_bwd_bnred``): writes ``dA`` and returns its BN partials as a
    ``_BnbPartials`` for ``_bn_bwd(pre=...)``, or None when not covered
    (``PDT_POOL_BNRED=0`` forces the separate passes)."""
    if os.environ.get("PDT_POOL_BNRED", "1") == "0" or (k, s, p) != (3, 2, 1) or not u.relu or u.mask is not None \
            or u.act is not None:
        return None
    lib = _load()
    N, C, H, W = u.N, u.Cout, u.g["Ho"], u.g["Wo"]
    Ho, Wo = dout.shape[2], dout.shape[3]
    blocks = min(int(os.environ.get("PDT_POOL_BNRED_BLOCKS", "8192")), N * ((H + 1) // 2))
    part = torch.empty(2 * blocks * C + lib.pdt_rows_reduce_workspace(blocks, C), dtype=torch.float32,
                       device=dout.device)
    rc = lib.pdt_maxpool_bwd_bnred(_p(dout), _p(idx), _p(dA), _p(u.y), _p(u.mean), _p(u.scale), _p(u.shift),
                                   _p(part), N, H, W, C, Ho, Wo, blocks, _s())
    if rc == NOT_APPLICABLE:
        return None
    _chk(rc, "maxpool_bwd_bnred")
    return _BnbPartials(part, blocks, u)


class _StemPool(torch.autograd.Function):
    """conv -> BN -> ReLU -> max-pool (the ResNet stem) with the BN apply folded into
    the max-pool: the full-resolution post-ReLU activation is never written or read.
    Backward: max-pool gradient -> BN backward (ReLU gate recomputed from y) -> weight
    gradient (and data gradient if the input needs one). PDT_STEM_POOL_BWD_FUSED=1 has
    the BN passes gather dA from the pool gradient and argmax instead (no
    full-resolution dA; measured no faster, so off by default)."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, conv, bna, k, s, p):
        if _s2d_ok(x, conv) and not ctx.needs_input_grad[0]:
            u = _unit_fwd_s2d(x, w, gamma, beta, bna)
        else:
            _, u = _unit_fwd(x, w, gamma, beta, None, conv, True, bna, apply=False)
        N, C, H, W = u.N, u.Cout, u.g["Ho"], u.g["Wo"]
        Ho = (H + 2 * p - k) // s + 1
        Wo = (W + 2 * p - k) // s + 1
        assert u.y.shape == (N, C, H, W) and u.y.is_contiguous(memory_format=torch.channels_last)
        out = _empty_cl(N, C, Ho, Wo, torch.bfloat16, u.y.device)
        idx = torch.empty(N * Ho * Wo * C, dtype=torch.uint8, device=u.y.device)
        _chk(_load().pdt_maxpool_fwd_affine(_p(u.y), _p(out), _p(idx), _p(u.scale), _p(u.shift), N, H, W, C, Ho, Wo,
                                            k, s, p, _s()), "maxpool_fwd_affine")
        ctx.u = u
        ctx.meta = (N, C, H, W, Ho, Wo, k, s, p)
        ctx.save_for_backward(u.x, u.y, idx)
        return out

    @staticmethod
    def backward(ctx, dout):
        u = ctx.u
        _, _, idx = ctx.saved_tensors
        N, C, H, W, Ho, Wo, k, s, p = ctx.meta
        dout = _cl(dout.to(torch.bfloat16))
        # off by default: measured equal to the composition (gathered reduce + apply 0.54 +
        # 0.66 ms vs maxpool_bwd + reduce + apply 0.44 + 0.31 + 0.46 ms at bs512, r59)
        if os.environ.get("PDT_STEM_POOL_BWD_FUSED", "0") == "1" and N * H * W * C < (1 << 34):
            dy, dgamma, dbeta = _bn_bwd_pool(dout, idx, u, k, s, p)
        else:
            dA = _empty_cl(N, C, H, W, torch.bfloat16, dout.device)
            s2d = u.g.get("s2d", False)
            fuse_red = s2d and ctx.needs_input_grad[1] and os.environ.get("PDT_STEM_WGRAD_BN", "1") == "1"
            pre = _pool_bwd_bnred(dout, idx, dA, u, k, s, p) if fuse_red else None
            if pre is None:
                _chk(_load().pdt_maxpool_bwd(_p(dout), _p(idx), _p(dA), N, H, W, C, Ho, Wo, k, s, p, _s()),
                     "maxpool_bwd")
            if fuse_red:
                # the stem's only consumer of dy is its weight gradient (no data gradient of the
                # image): the BN backward apply is formed in that GEMM's dY staging (tuned per shape)
                dgamma, dbeta, k1, k2, k3 = _bn_bwd(dA, u, False, coeffs_only=True, pre=pre)
                dw = _unit_dw_s2d(None, u, bn_dA=(dA, k1, k2, k3))
                del ctx.u
                return None, dw, dgamma, dbeta, None, None, None, None, None
            dy, _, dgamma, dbeta = _bn_bwd(dA, u, False)
        s2d = u.g.get("s2d", False)
        dx = _unit_dx(dy, u) if ctx.needs_input_grad[0] and not s2d else None
        dw = None
        if ctx.needs_input_grad[1]:
            dw = _unit_dw_s2d(dy, u) if s2d else _unit_dw(dy, u)
        del ctx.u
        return dx, dw, dgamma, dbeta, None, None, None, None, None


def stem_pool(x, conv: nn.Conv2d, bn: nn.BatchNorm2d, kernel_size=3, stride=2, padding=1):
    """max_pool2d(relu(bn(conv(x)))) as one node; None if the native path cannot run it."""
    if not supports_conv(x, conv) or conv.out_channels % 8:
        fallback("stem conv+bn+relu+maxpool", f"conv {tuple(conv.kernel_size)} on {tuple(x.shape)}")
        return None
    return _StemPool.apply(x, conv.weight, bn.weight, bn.bias, conv, _BNArgs(bn), kernel_size, stride, padding)


def max_pool2d(x, kernel_size=3, stride=2, padding=1):
    if x.dtype != torch.bfloat16 or x.shape[1] % 8:
        fallback("max_pool2d", f"{tuple(x.shape)} {x.dtype} (needs bf16, channels % 8 == 0)")
        return torch.nn.functional.max_pool2d(x, kernel_size, stride, padding)
    return _MaxPool.apply(x, kernel_size, stride, padding)


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _cl(x)
        N, C, H, W = x.shape
        y = torch.empty((N, C), dtype=torch.bfloat16, device=x.device)
        _chk(_load().pdt_avgpool_fwd(_p(x), _p(y), N, H * W, C, _s()), "avgpool_fwd")
        ctx.meta = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.meta
        dy = dy.to(torch.bfloat16).contiguous()
        dx = _empty_cl(N, C, H, W, torch.bfloat16, dy.device)
        _chk(_load().pdt_avgpool_bwd(_p(dy), _p(dx), N, H * W, C, _s()), "avgpool_bwd")
        return dx


def global_avg_pool(x):
    if x.dtype != torch.bfloat16 or x.shape[1] % 8:
        fallback("global_avg_pool", f"{tuple(x.shape)} {x.dtype} (needs bf16, channels % 8 == 0)")
        return torch.flatten(torch.nn.functional.adaptive_avg_pool2d(x, 1), 1)
    return _AvgPool.apply(x)


# =============================================================================
# linear (bf16 MFMA GEMM with bias / relu epilogue)
# =============================================================================
# -----------------------------------------------------------------------------
# Plain-GEMM backward of nn.Linear (reference op: /root/reference/model/model.py:19,21):
#   dX = dY W     -> the conv_nt NT kernel on the transposed bf16 weight W^T [K][Nout]
#                    (cast+transposed once per optimizer version, cached like the bf16 shadow)
#   dW = dY^T X   -> the split-K weight-gradient kernel (both operands K-outer, read
#                    through ds_read_b64_tr_b16), fp32 output for the optimizer
# Both are hand-written kernels with their own tile-variant tuning; there is no
# library-GEMM branch.
# -----------------------------------------------------------------------------
_WT: dict = {}


def bf16_weight_t(w: torch.Tensor) -> torch.Tensor:
    """bf16 W^T [K][Nout] of an fp32 [Nout][K] weight, cached per parameter version."""
    ent = _WT.get(id(w))
    if ent is not None and ent[0] == w._version and ent[1] == w.data_ptr() and _same_tensor(ent[3], w):
        return ent[2]
    Nout, K = w.shape
    wt = torch.empty((K, Nout), dtype=torch.bfloat16, device=w.device)
    _chk(_load().pdt_transpose_cast(_p(w.detach().float().contiguous()), _p(wt), Nout, K, _s()), "transpose")
    _WT[id(w)] = (w._version, w.data_ptr(), wt, _weak(w))
    return wt


def _linear_dgrad(dy2, w):
    Nout, K = w.shape
    Mrows = dy2.shape[0]
    wt = bf16_weight_t(w)
    dx = torch.empty((Mrows, K), dtype=torch.bfloat16, device=dy2.device)
    conv_nt(dy2, wt, dx, Hs=1, Ws=1, Cs=Nout, Nimg=Mrows, Hm=1, Wm=1, Ncol=K, K=Nout, ldb=Nout, sh=1, sw=1,
            oh0=0, ow0=0, dh=1, dw=1, nth=1, ntw=1, Ho=1, Wo=1, osh=1, osw=1, oph=0, opw=0, ldo=K)
    return dx


def _linear_wgrad(dy2, x2, w, with_bias=False, bias=None):
    """(dW fp32 [Nout][K], db fp32 [Nout] or None): db comes out of the same kernel."""
    Nout, K = w.shape
    dw = _grad_buf(w, (Nout, K), device=dy2.device)
    db = _grad_buf(bias, (Nout,), device=dy2.device) if with_bias else None
    conv_wgrad(dy2, x2, dw, M=dy2.shape[0], Mo=Nout, No=K, ldy=Nout, Hs=1, Ws=1, C=K, Hm=1, Wm=1, sh=1, sw=1,
               oh0=0, ow0=0, dh=1, dw=1, ntw=1, bias_out=db)
    return dw, db


def _linear_grads(dy2, x2, w, want_db, want_dw, bias=None):
    if want_dw:
        dw, db = _linear_wgrad(dy2, x2, w, with_bias=want_db, bias=bias)
        return dw, db
    return None, (colsum(dy2, dy2.shape[0], w.shape[0]) if want_db else None)


def _residual2d(residual, Mrows, Nout):
    if residual is None:
        return None
    r = residual.reshape(Mrows, Nout)
    assert r.dtype == torch.bfloat16, "residual stream must be bf16"
    return r.contiguous()


def _gemm_bf16(x2, wb, y, *, bias=None, act=None, aux=None, addend=None):
    """y[M, N] = x2[M, K] @ wb[N, K]^T (+bias, act) (+addend) on the conv_nt kernel."""
    Mrows, K = x2.shape
    Nout = wb.shape[0]
    conv_nt(x2, wb, y, Hs=1, Ws=1, Cs=K, Nimg=Mrows, Hm=1, Wm=1, Ncol=Nout, K=K, ldb=K, sh=1, sw=1, oh0=0,
            ow0=0, dh=1, dw=1, nth=1, ntw=1, Ho=1, Wo=1, osh=1, osw=1, oph=0, opw=0, ldo=Nout, bias=bias,
            act=act, aux=aux, addend=addend)
    return y


class _Linear(torch.autograd.Function):
    """y = act(x W^T + b) (+ residual): the residual add rides the GEMM epilogue and
    its gradient is dy itself (no add kernels either way)."""

    @staticmethod
    def forward(ctx, x, w, b, act, residual):
        ctx.bref = b  # the bias parameter: its gradient goes to its reducer slot
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(torch.bfloat16).contiguous()
        Mrows, K = x2.shape
        Nout = w.shape[0]
        wb = bf16_weight(w)
        y = torch.empty((Mrows, Nout), dtype=torch.bfloat16, device=x.device)
        z = torch.empty_like(y) if act == "gelu" else None  # pre-activation for GELU backward
        bias = b.float().contiguous() if b is not None else None
        _gemm_bf16(x2, wb, y, bias=bias, act=act, aux=z, addend=_residual2d(residual, Mrows, Nout))
        ctx.save_for_backward(x2, w, y if act == "relu" else z)
        ctx.meta = (shp, act, b is not None)
        return y.reshape(*shp[:-1], Nout)

    @staticmethod
    def backward(ctx, dy):
        x2, w, saved = ctx.saved_tensors
        shp, act, has_b = ctx.meta
        only = getattr(dy, "_pdt_f8g_only", None)
        if only is not None and (only is not ctx.fc or act is not None or not ctx.fp8_dgrad or not ctx.f8w):
            # the producer (the fp8 attention backward) wrote the e5m2 codes and the bias
            # gradient but not the bf16 values this configuration would read
            raise RuntimeError("this output gradient carries fp8 codes only (PDT_ATTN_BWD_Q8); its layer needs "
                               "the bf16 values: set PDT_ATTN_BWD_Q8_BF16=1 or PDT_ATTN_BWD_Q8=0")
        lib = _load()
        st = _s()
        Nout, K = w.shape
        dy2 = dy.reshape(-1, Nout).to(torch.bfloat16).contiguous()
        if act == "relu":
            dy2 = dy2 * (saved > 0)
        elif act == "gelu":
            dz = torch.empty_like(dy2)
            _chk(lib.pdt_gelu_bwd(_p(dy2), _p(saved), _p(dz), dz.numel(), st), "gelu_bwd")
            dy2 = dz
        Mrows = dy2.shape[0]
        dx = _linear_dgrad(dy2, w).reshape(*shp[:-1], K) if ctx.needs_input_grad[0] else None
        dw, db = _linear_grads(dy2, x2, w, has_b and ctx.needs_input_grad[2], ctx.needs_input_grad[1],
                               bias=ctx.bref)
        return dx, dw, db, None, (dy if ctx.needs_input_grad[4] else None)


# =============================================================================
# FP8 linear (OCP e4m3 forward operands, e5m2 output gradients) -- csrc/fp8.hip
# quantizes with per-tensor current scaling entirely on device; the GEMMs are
# the block-scaled fp8 MFMA instantiation of conv_nt (csrc/conv_igemm.hip,
# pdt_gemm_f8). Weight gradients stay bf16 (the wgrad kernel), as in common
# fp8 training recipes.
# =============================================================================
E4M3, E5M2 = 0, 1


def fp8_settings() -> dict:
    """The fp8 recipe actually in effect (read by the layers AND by bench.py's
    dtype label, so the label cannot drift from the code's defaults)."""
    return {"scaling": os.environ.get("PDT_FP8_SCALING", "delayed"),
            "dgrad": os.environ.get("PDT_FP8_DGRAD", "1") == "1",
            "attn": os.environ.get("PDT_FP8_ATTN", "1") == "1",
            "wgrad": os.environ.get("PDT_FP8_WGRAD", "1") == "1"}


def quantize_fp8(x: torch.Tensor, fmt: int = E4M3):
    """(q uint8 same shape, dq fp32[1]) with x ~= q.float() * dq (per-tensor scale)."""
    lib = _load()
    x = x.contiguous()
    assert x.dtype in (torch.bfloat16, torch.float32)
    n = x.numel()
    part = torch.empty(lib.pdt_amax_blocks(n), dtype=torch.float32, device=x.device)
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    dq = torch.empty(1, dtype=torch.float32, device=x.device)
    bf = int(x.dtype == torch.bfloat16)
    _chk(lib.pdt_amax_partial(_p(x), bf, n, _p(part), _s()), "amax")
    _chk(lib.pdt_cast_fp8(_p(x), bf, n, _p(part), fmt, _p(q), _p(dq), _s()), "cast_fp8")
    return q, dq


def quantize_fp8_delayed(x: torch.Tensor, meta: torch.Tensor | None, fmt: int = E4M3):
    """One-pass cast with delayed (amax-history) scaling; returns (q, dq, meta).

    ``meta`` is the tensor's scaling state (csrc/fp8.hip: scale, dq, amax,
    history); pass None on first use -- it is created and seeded with the
    exact amax of ``x`` (so the first step is current-scaled)."""
    lib = _load()
    x = x.contiguous()
    n = x.numel()
    bf = int(x.dtype == torch.bfloat16)
    if meta is None:
        meta = torch.zeros(lib.pdt_fp8_meta_words(), dtype=torch.float32, device=x.device)
        part = torch.empty(lib.pdt_amax_blocks(n), dtype=torch.float32, device=x.device)
        _chk(lib.pdt_amax_partial(_p(x), bf, n, _p(part), _s()), "amax")
        _chk(lib.pdt_fp8_meta_seed(_p(part), n, fmt, _p(meta), _s()), "fp8_meta_seed")
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    dq = torch.empty(1, dtype=torch.float32, device=x.device)  # this cast's dequant factor (stable)
    _chk(lib.pdt_cast_fp8_delayed(_p(x), bf, n, _p(meta), fmt, _p(q), _p(dq), _s()), "cast_fp8_delayed")
    return q, dq, meta


_F8W: dict = {}


def fp8_weight(w: torch.Tensor):
    """(wq [N][K] e4m3, wqt [K][N] e4m3, dq) of an fp32 [N][K] weight, cached per optimizer version."""
    ent = _F8W.get(id(w))
    if ent is not None and ent[0] == w._version and ent[1] == w.data_ptr() and _same_tensor(ent[3], w):
        return ent[2]
    lib = _load()
    src = w.detach().float().contiguous()
    N, K = src.shape
    part = torch.empty(lib.pdt_amax_blocks(src.numel()), dtype=torch.float32, device=w.device)
    wq = torch.empty((N, K), dtype=torch.uint8, device=w.device)
    wqt = torch.empty((K, N), dtype=torch.uint8, device=w.device)
    dq = torch.empty(1, dtype=torch.float32, device=w.device)
    st = _s()
    _chk(lib.pdt_amax_partial(_p(src), 0, src.numel(), _p(part), st), "amax")
    # both layouts (forward [N][K], data gradient [K][N]) from one read of the fp32 weight
    _chk(lib.pdt_cast_fp8_dual(_p(src), N, K, _p(part), _p(wq), _p(wqt), _p(dq), st), "cast_fp8_dual")
    val = (wq, wqt, dq)
    _F8W[id(w)] = (w._version, w.data_ptr(), val, _weak(w))
    return val


def _fc1_split(M, Hd, K) -> bool:
    """The MLP's fp8 fc1 as a plain GEMM (+bias) followed by one pass that writes gelu'(z), the
    e4m3 codes of gelu(z) and their amax (pdt_gelu_dual_cast_fp8), instead of one GEMM with that
    epilogue fused (act 4 + fp8 side output). Off by default: the dense ring's fused epilogue
    (csrc/gemm_ring.hip) measured faster than the split (ViT-B/16 fp8 bs 1024: 9 404 vs 9 175
    img/s with the fc2 data gradient below, same box, r5b). Tuned-table key
    ``fc1split:M,Hd,K`` (1 = split); PDT_FP8_FC1_SPLIT=0/1 forces either. (The hipBLASLt A/B
    of these plain GEMMs lives in ``scripts/probe_scaled_mm.py`` / ``scripts/bench_f8.py``,
    not in the product.)"""
    env = os.environ.get("PDT_FP8_FC1_SPLIT")
    if env is not None:
        return env == "1"
    return bool(_tuned().get(f"fc1split:{M},{Hd},{K}", 0))


def _fc1_split_forward(xq, w1q, a, z, aq, dqx, dqw1, bias1, meta, keep_a):
    """a <- x W1^T + b1 (plain fp8 GEMM), then z <- gelu'(a) (z None: not formed -- the caller keeps
    the pre-activation a), aq <- e4m3(gelu(a)), and (keep_a) a <- gelu(a) in place. Returns the
    codes' dequant factor (device [1])."""
    lib = _load()
    dqa = torch.empty(1, dtype=torch.float32, device=a.device)
    gemm_f8(xq, w1q, a, dqx, dqw1, fmt_a=E4M3, bias=bias1)
    _chk(lib.pdt_gelu_dual_cast_fp8(_p(a), a.numel(), _p(meta), E4M3, _p(aq), _p(z) if z is not None else None,
                                    _p(a) if keep_a else None, _p(dqa), _s()), "gelu_dual_cast_fp8")
    return dqa


def _fc2_dgrad_split_on() -> bool:
    """The MLP's fc2 data gradient as a plain GEMM (bf16 g W2) followed by one pass that
    multiplies by gelu'(z), casts to e5m2 and sums fc1's bias gradient
    (pdt_cast_fp8_gelu_grad_cs), instead of one GEMM with that epilogue (act 3 + e5m2 + column
    sums). Off by default (the fused ring epilogue is faster, see ``_fc1_split``);
    PDT_FC2_DGRAD_SPLIT=1 turns it on."""
    return os.environ.get("PDT_FC2_DGRAD_SPLIT", "0") == "1"


def _fc2_dgrad_split(gq, w2qt, dz, dqg, dqw2, z, dzq, gmeta, db):
    """dz <- g W2 (plain fp8 GEMM), then dzq <- e5m2(dz * gelu'(z)) and db <- column sums of dz * gelu'(z).
    Returns the codes' dequant factor (device [1])."""
    lib = _load()
    rows, cols = dz.shape
    gemm_f8(gq, w2qt, dz, dqg, dqw2, fmt_a=E5M2)
    nb = lib.pdt_cast_cs_bands(rows)
    cpart = torch.empty(nb * cols + lib.pdt_reduce_rows_work(nb, cols), dtype=torch.float32, device=dz.device)
    dq = torch.empty(1, dtype=torch.float32, device=dz.device)
    _chk(lib.pdt_cast_fp8_gelu_grad_cs(_p(dz), _p(z), rows, cols, _p(gmeta), E5M2, _p(dzq), _p(dq), _p(cpart),
                                       _p(db), _s()), "cast_fp8_gelu_grad_cs")
    return dq


def _fc1_keep_pre() -> bool:
    """Split fc1 with fp8 weight gradients: keep the GEMM's own pre-activation output for the
    backward (whose fc2 data-gradient epilogue then forms gelu'(z) itself, act 3) instead of
    writing gelu'(z) in the cast pass -- one bf16 [M, 4D] store fewer per block."""
    return os.environ.get("PDT_FC1_KEEP_PRE", "1") == "1"


def gemm_f8(a, b, out, dq_a, dq_b, *, fmt_a=E4M3, bias=None, act=0, aux=None, addend=None, variant=None,
            q8=None, colsum_out=None):
    """out[M, N] (bf16) = dq_a*dq_b * a[M, K] @ b[N, K]^T (+bias, act) (+ addend); a, b uint8 fp8
    codes. ``act=3``: GELU backward, out = (a @ b^T) * gelu'(addend).

    ``q8 = (codes, meta, fmt, only)``: the epilogue also writes the fp8 codes (format fmt) of
    the output for the NEXT fp8 GEMM with that GEMM's delayed scale ``meta`` and rolls its
    amax history (no separate quantisation pass); ``only`` skips the bf16 output. Returns
    the codes' dequant factor (device [1]) in that case, else ``out``. ``colsum_out`` (with q8,
    fp32 [N]): also the column sums of the final bf16 output (written or not), formed in the
    epilogue -- the bias gradient of the layer whose output gradient this GEMM produces."""
    M, K = a.shape
    N = b.shape[0]
    assert a.dtype == torch.uint8 and b.dtype == torch.uint8 and b.shape[1] == K and K % 128 == 0
    assert out.dtype == torch.bfloat16 and out.numel() == M * N and a.is_contiguous() and b.is_contiguous()
    lib = _load()
    if addend is not None:
        assert addend.dtype == torch.bfloat16 and addend.numel() == M * N and addend.is_contiguous()
    if q8 is None:
        args = lambda v: (_p(a), _p(b), _p(out), _p(bias), _p(dq_a), _p(dq_b), M, N, K, K, K, N, fmt_a, act,  # noqa
                          _p(aux), _p(addend), v, _s())
        nv = lib.pdt_gemm_f8_num_variants()
        if variant is None:
            # ",r": a residual addend in the epilogue (a different best tile); "f8c": the variant
            # set with the dense ring (ids 12 / 13)
            key = f"f8c:{M},{N},{K},{fmt_a},{act},{int(bias is not None)}" + (",r" if addend is not None and act == 0
                                                                               else "")
            variant = _autotune(key, nv, lambda v: lib.pdt_gemm_f8(*args(v)))
        if variant >= nv:
            variant = -1  # (a stale table entry: the built-in native choice)
        _chk_v(lib.pdt_gemm_f8(*args(variant)), "gemm_f8")
        return out
    codes, meta, qfmt, only = q8
    assert codes.dtype == torch.uint8 and codes.numel() == M * N and codes.is_contiguous()
    part = torch.empty(lib.pdt_gemm_f8_q8_part(M, N) + 1, dtype=torch.float32, device=a.device)
    dq = part[-1:]
    args = lambda v: (_p(a), _p(b), _p(out), _p(bias), _p(dq_a), _p(dq_b), M, N, K, K, K, N, fmt_a, act,  # noqa
                      _p(aux), _p(addend), v, _p(codes), _p(meta), _p(part), int(qfmt), int(only), _p(dq), _s())
    if variant is None:
        key = f"f8c:{M},{N},{K},{fmt_a},{act},{int(bias is not None)},q{qfmt}{int(only)}" + \
            (",cs" if colsum_out is not None else "")
        table = _tuned()
        if key in table:
            variant = int(table[key])
        else:
            # (tuning launches roll the history too: tune on a scratch copy of the state)
            scratch = meta.clone()
            targs = lambda v: args(v)[:17] + (_p(codes), _p(scratch)) + args(v)[19:]  # noqa: E731
            variant = _autotune(key, lib.pdt_gemm_f8_num_variants(), lambda v: lib.pdt_gemm_f8_q8(*targs(v)))
    if colsum_out is not None:
        assert colsum_out.dtype == torch.float32 and colsum_out.numel() == N and colsum_out.is_contiguous()
        if variant == 7 or variant < 0:  # the direct-store tile has no staged epilogue
            variant = 10
        ntm = -(-M // lib.pdt_gemm_f8_bm(variant))
        cpart = torch.empty(ntm * N + lib.pdt_reduce_rows_work(ntm, N), dtype=torch.float32, device=a.device)
        _chk_v(lib.pdt_gemm_f8_q8_cs(*args(variant)[:-1], _p(cpart), _s()), "gemm_f8_q8_cs")
        _chk(lib.pdt_wgrad_reduce_rows(_p(cpart), _p(colsum_out), ntm, N, 1.0, 0, _p(cpart[ntm * N:]), _s()),
             "colsum rows")
        return dq
    _chk_v(lib.pdt_gemm_f8_q8(*args(variant)), "gemm_f8_q8")
    return dq


def _wgrad_f8_launch(lib, dyq, xq, dq_dy, dq_x, dy16, dw, db, v):
    M, Mo = dyq.shape
    No = xq.shape[1]
    kps = c_int(0)
    splits = lib.pdt_wgrad_f8_plan(M, Mo, No, v, ctypes.byref(kps))
    slab = torch.empty(lib.pdt_wgrad_f8_workspace(splits, Mo, No), dtype=torch.float32, device=dyq.device)
    _chk(lib.pdt_linear_wgrad_f8(_p(dyq), _p(xq), _p(dq_dy), _p(dq_x), _p(dy16), _p(slab), _p(dw), _p(db), M, Mo, No,
                                 Mo, No, splits, kps.value, 0, int(v), _s()), "linear_wgrad_f8")


def linear_wgrad_f8(dyq, xq, dq_dy, dq_x, dy16=None, with_bias=False, variant=None, w=None, b=None):
    """(dW fp32 [Nout][K], db fp32 [Nout] or None) of nn.Linear from the fp8 codes the
    data-gradient and forward GEMMs consumed: dyq [M][Nout] e5m2, xq [M][K] e4m3, device
    dequant scales. db = column sums of the bf16 ``dy16`` (csrc/wgrad_f8.hip)."""
    M, Nout = dyq.shape
    K = xq.shape[1]
    assert dyq.dtype == torch.uint8 and xq.dtype == torch.uint8 and xq.shape[0] == M
    assert dyq.is_contiguous() and xq.is_contiguous() and Nout % 16 == 0 and K % 16 == 0
    if with_bias:
        assert dy16 is not None and dy16.dtype == torch.bfloat16 and dy16.shape == (M, Nout) and dy16.is_contiguous()
    lib = _load()
    dw = _grad_buf(w, (Nout, K)) if w is not None else torch.empty((Nout, K), dtype=torch.float32,
                                                                  device=dyq.device)
    db = (_grad_buf(b, (Nout,)) if b is not None else torch.empty(Nout, dtype=torch.float32, device=dyq.device)) \
        if with_bias else None
    if variant is None:
        key = f"wg8:{M},{Nout},{K}"
        table = _tuned()
        if key in table:
            variant = int(table[key])
        elif not _tune_allowed():
            variant = 0
        else:
            best = _time_variants(lib.pdt_wgrad_f8_num_variants(),
                                  lambda v: _wgrad_f8_launch(lib, dyq, xq, dq_dy, dq_x, None, dw, None, v) or 0)
            table[key] = best
            _save_tuned()
            variant = best
    _wgrad_f8_launch(lib, dyq, xq, dq_dy, dq_x, dy16 if with_bias else None, dw, db, variant)
    return dw, db


def _quant_grad_db(g2, owner, attr, bias):
    """(e5m2 codes, dequant, bias gradient) of a bf16 [rows][cols] output gradient in ONE pass
    (pdt_cast_fp8_delayed_cs: the delayed-scaling cast that also sums the columns it reads),
    or None when that path does not apply (current scaling, no history yet, PDT_CAST_DB=0)."""
    meta = getattr(owner, attr, None)
    if meta is None or fp8_settings()["scaling"] != "delayed" or os.environ.get("PDT_CAST_DB", "1") != "1":
        return None
    rows, cols = g2.shape
    if cols % 8:
        return None
    lib = _load()
    nb = lib.pdt_cast_cs_bands(rows)
    q = torch.empty((rows, cols), dtype=torch.uint8, device=g2.device)
    dq = torch.empty(1, dtype=torch.float32, device=g2.device)
    cpart = torch.empty(nb * cols + lib.pdt_reduce_rows_work(nb, cols), dtype=torch.float32, device=g2.device)
    db = _grad_buf(bias, (cols,))
    _chk(lib.pdt_cast_fp8_delayed_cs(_p(g2), rows, cols, _p(meta), E5M2, _p(q), _p(dq), _p(cpart), _p(db), _s()),
         "cast_fp8_delayed_cs")
    return q, dq, db


def _pre_bias_grad(g, owner):
    """The bias gradient of ``owner`` if the producer of its output gradient ``g`` (a LayerNorm
    backward, :func:`_ln_fork_backward`) already formed it, else None."""
    pre = getattr(g, "_pdt_db", None) if g is not None else None
    if pre is None or pre[1] is not owner:
        return None
    # dropped from ``g``: a LayerNorm's dx also feeds the residual branch, so it outlives this
    # backward, and a second reference to the bias gradient (a reducer slot view) would make
    # autograd clone it instead of adopting it as ``bias.grad`` (and the reducer copy it back)
    del g._pdt_db
    return pre[0]


def _fp8_wgrad_on() -> bool:
    return fp8_settings()["wgrad"]


def _quant_act(x2, owner, attr="_pdt_fp8_meta"):
    """e4m3 codes + dequant scale of a bf16 activation under the configured scaling
    (delayed: amax history kept on ``owner``)."""
    if fp8_settings()["scaling"] == "current":
        return quantize_fp8(x2, E4M3)
    q, dq, meta = quantize_fp8_delayed(x2, getattr(owner, attr, None), E4M3)
    setattr(owner, attr, meta)
    return q, dq


def _quant_grad(g2, owner, attr, src=None):
    """e5m2 codes + dequant scale of an output gradient for the fp8 data-gradient GEMM.
    Delayed scaling (the default) is one fused cast+amax pass with the history kept on
    ``owner``; current scaling needs a separate amax pass over the gradient first.
    ``src``: the gradient tensor as received -- if its producer (the LayerNorm backward,
    ``ln_fork(grad_fp8_for=owner)``) already wrote the codes, they are used as they are."""
    pre = getattr(src, "_pdt_f8g", None) if src is not None else None
    if pre is not None and pre[2] is owner:
        return pre[0].view(g2.shape), pre[1]
    if fp8_settings()["scaling"] == "current":
        return quantize_fp8(g2, E5M2)
    q, dq, meta = quantize_fp8_delayed(g2, getattr(owner, attr, None), E5M2)
    setattr(owner, attr, meta)
    return q, dq


class _LinearF8(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, fc, residual):
        ctx.bref = b
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(torch.bfloat16).contiguous()
        Mrows, K = x2.shape
        Nout = w.shape[0]
        cfg = fp8_settings()
        pre = _prequant(x, fc)
        xq, dqx = pre if pre is not None else _quant_act(x2, fc)
        wq, _, dqw = fp8_weight(w)
        y = torch.empty((Mrows, Nout), dtype=torch.bfloat16, device=x.device)
        z = torch.empty_like(y) if act == "gelu" else None
        bias = b.float().contiguous() if b is not None else None
        gemm_f8(xq, wq, y, dqx, dqw, bias=bias, act=ACT[act], aux=z, addend=_residual2d(residual, Mrows, Nout))
        # fp8 weight gradient (needs the e5m2 dY codes of the fp8 data gradient): keep the
        # e4m3 input codes + their dequant scale instead of the bf16 input
        ctx.f8w = cfg["dgrad"] and cfg["wgrad"] and K % 16 == 0 and Nout % 16 == 0
        if ctx.f8w:
            ctx.xq, ctx.dqx = xq, dqx
            ctx.save_for_backward(None, w, y if act == "relu" else z)
        else:
            ctx.save_for_backward(x2, w, y if act == "relu" else z)
        ctx.meta = (shp, act, b is not None)
        ctx.fc = fc
        # e5m2 data-gradient GEMM (default on; PDT_FP8_DGRAD=0 keeps it bf16)
        ctx.fp8_dgrad = cfg["dgrad"]
        return y.reshape(*shp[:-1], Nout)

    @staticmethod
    def backward(ctx, dy):
        x2, w, saved = ctx.saved_tensors
        shp, act, has_b = ctx.meta
        only = getattr(dy, "_pdt_f8g_only", None)
        if only is not None and (only is not ctx.fc or act is not None or not ctx.fp8_dgrad or not ctx.f8w):
            # the producer (the fp8 attention backward) wrote the e5m2 codes and the bias
            # gradient but not the bf16 values this configuration would read
            raise RuntimeError("this output gradient carries fp8 codes only (PDT_ATTN_BWD_Q8); its layer needs "
                               "the bf16 values: set PDT_ATTN_BWD_Q8_BF16=1 or PDT_ATTN_BWD_Q8=0")
        lib = _load()
        Nout, K = w.shape
        dy2 = dy.reshape(-1, Nout).to(torch.bfloat16).contiguous()
        if act == "relu":
            dy2 = dy2 * (saved > 0)
        elif act == "gelu":
            dz = torch.empty_like(dy2)
            _chk(lib.pdt_gelu_bwd(_p(dy2), _p(saved), _p(dz), dz.numel(), _s()), "gelu_bwd")
            dy2 = dz
        Mrows = dy2.shape[0]
        need = ctx.needs_input_grad
        dx = None
        dyq = dqdy = None
        cast_db = None
        if ctx.fp8_dgrad and (need[0] or (ctx.f8w and need[1])):
            pre = getattr(dy, "_pdt_f8g", None) if act is None else None
            if act is None and has_b and need[2] and ctx.f8w and need[1] and (pre is None or pre[2] is not ctx.fc):
                cast_db = _quant_grad_db(dy2, ctx.fc, "_pdt_fp8_gmeta", ctx.bref)
            if cast_db is not None:
                dyq, dqdy = cast_db[0], cast_db[1]
            else:
                dyq, dqdy = _quant_grad(dy2, ctx.fc, "_pdt_fp8_gmeta", src=dy if act is None else None)
        if need[0]:
            if ctx.fp8_dgrad:
                _, wqt, dqw = fp8_weight(w)
                dx = torch.empty((Mrows, K), dtype=torch.bfloat16, device=dy.device)
                gemm_f8(dyq, wqt, dx, dqdy, dqw, fmt_a=E5M2)
            else:
                dx = _linear_dgrad(dy2, w)
            dx = dx.reshape(*shp[:-1], K)
        want_db = has_b and need[2]
        pre_db = _pre_bias_grad(dy, ctx.fc) if act is None and want_db else None
        if pre_db is None and cast_db is not None:
            pre_db = cast_db[2]
        if ctx.f8w and need[1]:
            dw, db = linear_wgrad_f8(dyq, ctx.xq, dqdy, ctx.dqx, dy16=dy2, with_bias=want_db and pre_db is None, w=w,
                                     b=ctx.bref)
            if pre_db is not None:
                db = pre_db
        elif ctx.f8w:
            dw, db = None, (colsum(dy2, Mrows, Nout) if want_db else None)
        else:
            dw, db = _linear_grads(dy2, x2, w, want_db, need[1], bias=ctx.bref)
        ctx.xq = ctx.dqx = None
        return dx, dw, db, None, None, (dy if need[5] else None)


def linear(x, fc: nn.Linear, act=None, fp8=False, residual=None):
    """act(x W^T + b) (+ residual, added in the GEMM epilogue)."""
    K = fc.in_features
    N = fc.out_features
    if K % 8 or N % 8 or act not in (None, "relu", "gelu") or (residual is not None and (
            residual.dtype != torch.bfloat16 or residual.shape[:-1] != x.shape[:-1] or residual.shape[-1] != N)):
        fallback("linear", f"{K}->{N} act={act} (needs K, N % 8 == 0, act in relu/gelu/None, bf16 residual)")
        from .fused import _torch_linear
        y = _torch_linear(x, fc, act)
        return y if residual is None else y + residual
    if fp8 and K % 128 == 0 and N % 128 == 0:
        return _LinearF8.apply(x, fc.weight, fc.bias, act, fc, residual)
    return _Linear.apply(x, fc.weight, fc.bias, act, residual)


# -----------------------------------------------------------------------------
# Transformer MLP as one autograd node: fc1 (+bias, GELU in the epilogue, the
# pre-activation z kept as the aux output) -> fc2 (+bias, + residual in the
# epilogue). Backward: the fc2 data gradient's epilogue applies GELU'(z) (conv_nt
# act 3), so dL/dz comes out of that GEMM -- no gelu_bwd pass -- and both bias
# gradients come out of the weight-gradient kernels. fp8 (e4m3 forward operands,
# e5m2 output gradients when PDT_FP8_DGRAD=1) or bf16 GEMMs.
# -----------------------------------------------------------------------------
class _Mlp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual, mlp, fp8):
        ctx.brefs = (b1, b2)
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(torch.bfloat16).contiguous()
        Mrows, K = x2.shape
        Hd, Nout = w1.shape[0], w2.shape[0]
        dev = x.device
        a = torch.empty((Mrows, Hd), dtype=torch.bfloat16, device=dev)
        z = None
        out = torch.empty((Mrows, Nout), dtype=torch.bfloat16, device=dev)
        res = _residual2d(residual, Mrows, Nout)
        bias1, bias2 = b1.float().contiguous(), b2.float().contiguous()
        cfg = fp8_settings()
        f8w = fp8 and cfg["dgrad"] and cfg["wgrad"]
        dual = _gelu_dual()
        act1 = ACT_GELU_DUAL if dual else ACT["gelu"]  # z holds gelu'(fc1 pre-activation) when dual
        act2 = ACT_MUL if dual else ACT_GELU_GRAD      # the fc2 data gradient's epilogue
        if fp8:
            pre = _prequant(x, mlp.fc1)
            xq, dqx = pre if pre is not None else _quant_act(x2, mlp.fc1)
            w1q, _, dqw1 = fp8_weight(w1)
            meta2 = getattr(mlp.fc2, "_pdt_fp8_meta", None) if cfg["scaling"] == "delayed" else None
            if meta2 is not None:  # fc1's epilogue writes fc2's e4m3 input (bf16 a only if a bf16 wgrad needs it)
                aq = torch.empty((Mrows, Hd), dtype=torch.uint8, device=dev)
                dqa = None
                if dual and _fc1_split(Mrows, Hd, K):
                    pre = f8w and _fc1_keep_pre()
                    z = None if pre else torch.empty_like(a)
                    dqa = _fc1_split_forward(xq, w1q, a, z, aq, dqx, dqw1, bias1, meta2, keep_a=not f8w)
                    if pre:  # a holds the pre-activation (its gelu lives only as the e4m3 codes)
                        z, act2 = a, ACT_GELU_GRAD
                if dqa is None:
                    z = torch.empty_like(a)
                    dqa = gemm_f8(xq, w1q, a, dqx, dqw1, bias=bias1, act=act1, aux=z, q8=(aq, meta2, E4M3, f8w))
            else:
                z = torch.empty_like(a)
                gemm_f8(xq, w1q, a, dqx, dqw1, bias=bias1, act=act1, aux=z)
                aq, dqa = _quant_act(a, mlp.fc2)
            w2q, _, dqw2 = fp8_weight(w2)
            gemm_f8(aq, w2q, out, dqa, dqw2, bias=bias2, addend=res)
        else:
            z = torch.empty_like(a)
            _gemm_bf16(x2, bf16_weight(w1), a, bias=bias1, act=act1, aux=z)
            _gemm_bf16(a, bf16_weight(w2), out, bias=bias2, addend=res)
        if f8w:  # fp8 weight gradients: the e4m3 GEMM inputs replace the bf16 ones in the saved state
            ctx.f8 = (xq, dqx, aq, dqa)
            ctx.save_for_backward(None, None, z, w1, w2)
        else:
            ctx.f8 = None
            ctx.save_for_backward(x2, a, z, w1, w2)
        ctx.shp, ctx.fp8, ctx.mlp = shp, fp8, mlp
        ctx.act2 = act2
        ctx.fp8_dgrad = fp8 and cfg["dgrad"]
        return out.reshape(*shp[:-1], Nout)

    @staticmethod
    def backward(ctx, g):
        x2, a, z, w1, w2 = ctx.saved_tensors
        need = ctx.needs_input_grad
        Mrows = z.shape[0]
        Hd, Nout = w1.shape[0], w2.shape[0]
        K = w1.shape[1]
        g2 = g.reshape(Mrows, Nout).to(torch.bfloat16).contiguous()
        dz = torch.empty((Mrows, Hd), dtype=torch.bfloat16, device=g.device)
        f8 = ctx.f8
        dzq = dqdz = pre_db1 = None
        if ctx.fp8_dgrad:
            gq, dqg = _quant_grad(g2, ctx.mlp.fc2, "_pdt_fp8_gmeta", src=g)
            _, w2qt, dqw2 = fp8_weight(w2)
            gmeta1 = getattr(ctx.mlp.fc1, "_pdt_fp8_gmeta", None) if fp8_settings()["scaling"] == "delayed" \
                else None
            if gmeta1 is not None:  # the epilogue also writes fc1's e5m2 output gradient (bf16 dz: bias grad)
                dzq = torch.empty((Mrows, Hd), dtype=torch.uint8, device=g.device)
                if f8 is not None and need[1] and need[2] and os.environ.get("PDT_F8_DB_EPI", "1") == "1":
                    # fc1's bias gradient = column sums of dz formed in this epilogue: the bf16 dz
                    # (only ever read for it) is not written at all
                    pre_db1 = _grad_buf(ctx.brefs[0], (Hd,))
                    if ctx.act2 == ACT_GELU_GRAD and _fc2_dgrad_split_on():  # z: the pre-activation
                        dqdz = _fc2_dgrad_split(gq, w2qt, dz, dqg, dqw2, z, dzq, gmeta1, pre_db1)
                    if dqdz is None:
                        dqdz = gemm_f8(gq, w2qt, dz, dqg, dqw2, fmt_a=E5M2, act=ctx.act2, addend=z,
                                       q8=(dzq, gmeta1, E5M2, True), colsum_out=pre_db1)
                else:
                    dqdz = gemm_f8(gq, w2qt, dz, dqg, dqw2, fmt_a=E5M2, act=ctx.act2, addend=z,
                                   q8=(dzq, gmeta1, E5M2, False))
            else:
                gemm_f8(gq, w2qt, dz, dqg, dqw2, fmt_a=E5M2, act=ctx.act2, addend=z)
        else:
            _gemm_bf16(g2, bf16_weight_t(w2), dz, act=ctx.act2, addend=z)  # dz = (g W2) * gelu'(z)
        pre_db2 = _pre_bias_grad(g, ctx.mlp.fc2) if need[4] else None
        if f8 is not None:
            dw2, db2 = linear_wgrad_f8(gq, f8[2], dqg, f8[3], dy16=g2, with_bias=need[4] and pre_db2 is None, w=w2,
                                       b=ctx.brefs[1]) if need[3] \
                else (None, colsum(g2, Mrows, Nout) if need[4] and pre_db2 is None else None)
            if pre_db2 is not None:
                db2 = pre_db2
        else:
            dw2, db2 = _linear_grads(g2, a, w2, need[4], need[3], bias=ctx.brefs[1])
        dx = None
        if dzq is None and ctx.fp8_dgrad and (need[0] or (f8 is not None and need[1])):
            dzq, dqdz = _quant_grad(dz, ctx.mlp.fc1, "_pdt_fp8_gmeta")
        if need[0]:
            dx = torch.empty((Mrows, K), dtype=torch.bfloat16, device=g.device)
            if ctx.fp8_dgrad:
                _, w1qt, dqw1 = fp8_weight(w1)
                gemm_f8(dzq, w1qt, dx, dqdz, dqw1, fmt_a=E5M2)
            else:
                _gemm_bf16(dz, bf16_weight_t(w1), dx)
            dx = dx.reshape(ctx.shp)
        if f8 is not None:
            dw1, db1 = linear_wgrad_f8(dzq, f8[0], dqdz, f8[1], dy16=dz, with_bias=need[2] and pre_db1 is None,
                                       w=w1, b=ctx.brefs[0]) if need[1] \
                else (None, colsum(dz, Mrows, Hd) if need[2] else None)
            if pre_db1 is not None:
                db1 = pre_db1
        else:
            dw1, db1 = _linear_grads(dz, x2, w1, need[2], need[1], bias=ctx.brefs[0])
        ctx.f8 = None
        return dx, dw1, db1, dw2, db2, (g if need[5] else None), None, None


def mlp(x, m, fp8=False, residual=None):
    """fc2(gelu(fc1(x))) (+ residual) for an Mlp module with fc1 / fc2 (ViT)."""
    fc1, fc2 = m.fc1, m.fc2
    K, Hd, N = fc1.in_features, fc1.out_features, fc2.out_features
    ok = (K % 8 == 0 and Hd % 8 == 0 and N % 8 == 0 and fc2.in_features == Hd and fc1.bias is not None
          and fc2.bias is not None and (residual is None or (residual.dtype == torch.bfloat16
                                                            and residual.shape[:-1] == x.shape[:-1]
                                                            and residual.shape[-1] == N)))
    use8 = fp8 and K % 128 == 0 and Hd % 128 == 0 and N % 128 == 0
    if not ok:
        y = linear(linear(x, fc1, act="gelu", fp8=fp8), fc2, fp8=fp8)
        return y if residual is None else y + residual
    return _Mlp.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, residual, m, use8)


# =============================================================================
# LayerNorm (bf16 activations, fp32 affine params)
# =============================================================================
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, eps):
        ctx.refs = (g, b)  # the affine parameters: their gradients go to their reducer slots
        shp = x.shape
        D = shp[-1]
        x2 = x.reshape(-1, D).to(torch.bfloat16).contiguous()
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        stats = torch.empty((2, rows), dtype=torch.float32, device=x.device)
        gf = g.float().contiguous()
        bf = b.float().contiguous()
        _chk(_load().pdt_ln_fwd(_p(x2), _p(gf), _p(bf), _p(y), _p(stats[0]), _p(stats[1]), rows, D, float(eps),
                                _s()), "ln_fwd")
        ctx.save_for_backward(x2, gf, stats)
        ctx.shp = shp
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, gf, stats = ctx.saved_tensors
        rows, D = x2.shape
        lib = _load()
        dy2 = dy.reshape(rows, D).to(torch.bfloat16).contiguous()
        dx = torch.empty_like(x2)
        blocks = lib.pdt_ln_bwd_blocks(rows)
        part = torch.empty(2 * blocks * D, dtype=torch.float32, device=dy.device)
        dg, db = _grad_buf(ctx.refs[0], (D,)), _grad_buf(ctx.refs[1], (D,))
        _chk(lib.pdt_ln_bwd(_p(dy2), _p(x2), _p(gf), _p(stats[0]), _p(stats[1]), _p(dx), _p(dg), _p(db), _p(part),
                            rows, D, 0, None, _s()), "ln_bwd")
        return dx.reshape(ctx.shp), dg, db, None


def layer_norm(x, ln):
    D = ln.normalized_shape[-1]
    if len(ln.normalized_shape) != 1 or D not in (256, 512, 768, 1024) or not ln.elementwise_affine:
        fallback("layer_norm", f"normalized_shape {tuple(ln.normalized_shape)} (kernels: D in 256/512/768/1024, affine)")
        return ln(x)
    return _LayerNorm.apply(x, ln.weight, ln.bias, ln.eps)


class _LNFork(torch.autograd.Function):
    """(x, LayerNorm(x)) for a pre-norm residual block: the pass-through output feeds
    the block's residual add (a GEMM epilogue), so backward receives the residual
    gradient and the normalised branch's gradient together and sums them inside
    the LayerNorm backward kernel (no add pass)."""

    @staticmethod
    def forward(ctx, x, g, b, eps, f8meta, f8box, grad_owner, codes_only=False):
        ctx.refs = (g, b)
        shp = x.shape
        D = shp[-1]
        x2 = x.reshape(-1, D).contiguous()
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        stats = torch.empty((2, rows), dtype=torch.float32, device=x.device)
        gf = g.float().contiguous()
        lib = _load()
        bf = b.float().contiguous()
        if f8meta is not None:  # also emit the next fp8 GEMM's e4m3 input (delayed scale f8meta)
            q = torch.empty((rows, D), dtype=torch.uint8, device=x.device)
            part = torch.empty(lib.pdt_ln_fwd_f8_blocks(rows) + 1, dtype=torch.float32, device=x.device)
            dq = part[-1:]  # the codes' dequant factor (written by the history roll)
            # codes_only: the bf16 output is not written (y stays uninitialised; see _ln_codes_only)
            _chk(lib.pdt_ln_fwd_f8(_p(x2), _p(gf), _p(bf), None if codes_only else _p(y), _p(stats[0]),
                                   _p(stats[1]), rows, D, float(eps), _p(q), _p(f8meta), _p(part), _p(dq), _s()),
                 "ln_fwd_f8")
            f8box.append((q, dq))
        else:
            _chk(lib.pdt_ln_fwd(_p(x2), _p(gf), _p(bf), _p(y), _p(stats[0]), _p(stats[1]), rows, D, float(eps),
                                _s()), "ln_fwd")
        ctx.save_for_backward(x2, gf, stats)
        ctx.shp = shp
        ctx.grad_owner = grad_owner
        return x.view_as(x), y.reshape(shp)

    @staticmethod
    def backward(ctx, g_res, dy):
        if dy is None:
            return g_res, None, None, None, None, None, None, None
        dx, dg, db = _ln_fork_backward(ctx, g_res, dy)
        return dx, dg, db, None, None, None, None, None


def _ln_fork_backward(ctx, g_res, dy):
    """LayerNorm backward of a fork (x -> (x, LN(x))) with the residual gradient g_res summed
    in: (dx, dgamma, dbeta); dx carries the e5m2 codes for ctx.grad_owner (``_pdt_f8g``) when
    that fp8 layer's gradient history exists."""
    x2, gf, stats = ctx.saved_tensors
    rows, D = x2.shape
    lib = _load()
    dev = x2.device
    dy2 = dy.reshape(rows, D).to(torch.bfloat16).contiguous()
    add = g_res.reshape(rows, D).to(torch.bfloat16).contiguous() if g_res is not None else None
    dx = torch.empty_like(x2)
    blocks = lib.pdt_ln_bwd_blocks(rows)
    part = torch.empty(2 * blocks * D, dtype=torch.float32, device=dev)
    dg, db = _grad_buf(ctx.refs[0], (D,)), _grad_buf(ctx.refs[1], (D,))
    owner = ctx.grad_owner
    gmeta = getattr(owner, "_pdt_fp8_gmeta", None) if owner is not None else None
    if gmeta is not None and fp8_settings()["scaling"] == "delayed":
        # also the e5m2 codes of dx for the fp8 GEMM that consumes this gradient
        codes = torch.empty((rows, D), dtype=torch.uint8, device=dev)
        qpart = torch.empty(blocks + 1, dtype=torch.float32, device=dev)
        dq = qpart[-1:]
        bias = getattr(owner, "bias", None)
        if bias is not None and bias.requires_grad and os.environ.get("PDT_LN_DB", "1") == "1":
            # the producer's bias gradient = column sums of dx, formed here (the weight-gradient
            # kernel of that layer would re-read dx for them); picked up through ``_pdt_db``
            pdb = _grad_buf(bias, (D,))
            cpart = torch.empty(blocks * D + lib.pdt_reduce_rows_work(blocks, D), dtype=torch.float32, device=dev)
            _chk(lib.pdt_ln_bwd_f8_db(_p(dy2), _p(x2), _p(gf), _p(stats[0]), _p(stats[1]), _p(dx), _p(dg), _p(db),
                                      _p(part), rows, D, 0, _p(add), _p(codes), _p(gmeta), _p(qpart), _p(dq),
                                      _p(cpart), _p(pdb), 0, _s()), "ln_bwd_f8_db")
        else:
            pdb = None
            _chk(lib.pdt_ln_bwd_f8(_p(dy2), _p(x2), _p(gf), _p(stats[0]), _p(stats[1]), _p(dx), _p(dg), _p(db),
                                   _p(part), rows, D, 0, _p(add), _p(codes), _p(gmeta), _p(qpart), _p(dq), _s()),
                 "ln_bwd_f8")
        out = dx.reshape(ctx.shp)
        out._pdt_f8g = (codes, dq, owner)
        if pdb is not None:
            out._pdt_db = (pdb, owner)
        return out, dg, db
    _chk(lib.pdt_ln_bwd(_p(dy2), _p(x2), _p(gf), _p(stats[0]), _p(stats[1]), _p(dx), _p(dg), _p(db), _p(part),
                        rows, D, 0, _p(add), _s()), "ln_bwd")
    return dx.reshape(ctx.shp), dg, db


class _LNAddFork(torch.autograd.Function):
    """(s, LayerNorm(s)) with s = y + r: the pre-norm block's residual add done by the
    LayerNorm kernel (it reads y and r, writes s) instead of the epilogue of the GEMM that
    produced y -- so that GEMM is a plain ring GEMM (no residual addend in its epilogue). Backward
    as _LNFork; y and r both receive the summed gradient."""

    @staticmethod
    def forward(ctx, y, r, g, b, eps, f8meta, f8box, grad_owner, codes_only=False):
        ctx.refs = (g, b)
        shp = y.shape
        D = shp[-1]
        y2 = y.reshape(-1, D).contiguous()
        r2 = r.reshape(-1, D).to(torch.bfloat16).contiguous()
        rows = y2.shape[0]
        xs = torch.empty_like(y2)
        h = torch.empty_like(y2)
        stats = torch.empty((2, rows), dtype=torch.float32, device=y.device)
        gf, bf = g.float().contiguous(), b.float().contiguous()
        lib = _load()
        if f8meta is not None:
            q = torch.empty((rows, D), dtype=torch.uint8, device=y.device)
            part = torch.empty(lib.pdt_ln_fwd_f8_blocks(rows) + 1, dtype=torch.float32, device=y.device)
            dq = part[-1:]
            _chk(lib.pdt_ln_add_fwd(_p(y2), _p(r2), _p(xs), _p(gf), _p(bf), None if codes_only else _p(h),
                                    _p(stats[0]), _p(stats[1]), rows, D, float(eps), _p(q), _p(f8meta), _p(part),
                                    _p(dq), _s()), "ln_add_fwd_f8")
            f8box.append((q, dq))
        else:
            _chk(lib.pdt_ln_add_fwd(_p(y2), _p(r2), _p(xs), _p(gf), _p(bf), _p(h), _p(stats[0]), _p(stats[1]), rows, D,
                                    float(eps), None, None, None, None, _s()), "ln_add_fwd")
        ctx.save_for_backward(xs, gf, stats)
        ctx.shp = shp
        ctx.grad_owner = grad_owner
        return xs.reshape(shp), h.reshape(shp)

    @staticmethod
    def backward(ctx, g_res, dy):
        if dy is None:
            return g_res, g_res, None, None, None, None, None, None, None
        dx, dg, db = _ln_fork_backward(ctx, g_res, dy)
        return dx, dx, dg, db, None, None, None, None, None


def ln_add_fork(y, r, ln, fp8_for=None, grad_fp8_for=None):
    """(y + r, ln(y + r)) -- :func:`ln_fork` with the residual add done by the LayerNorm kernel
    (``grad_fp8_for``: the fp8 layer that produced ``y``)."""
    D = ln.normalized_shape[-1]
    if (len(ln.normalized_shape) != 1 or D not in (256, 512, 768, 1024) or not ln.elementwise_affine
            or y.dtype != torch.bfloat16 or r.shape != y.shape):
        return ln_fork(y + r.to(y.dtype), ln, fp8_for, grad_fp8_for)
    meta = None
    if fp8_for is not None and fp8_settings()["scaling"] == "delayed" and D % 128 == 0:
        meta = getattr(fp8_for, "_pdt_fp8_meta", None)
    box: list = []
    if os.environ.get("PDT_FP8_LN_GRAD", "1") == "0":
        grad_fp8_for = None
    only = meta is not None and _ln_codes_only(fp8_for)
    xo, h = _LNAddFork.apply(y, r, ln.weight, ln.bias, ln.eps, meta, box, grad_fp8_for, only)
    if box:
        h._pdt_f8 = (box[0][0], box[0][1], fp8_for)
        if only:
            h._pdt_f8_only = True
    return xo, h


def ln_fork(x, ln, fp8_for=None, grad_fp8_for=None):
    """(x, ln(x)) with the residual gradient summed in LayerNorm's backward (see _LNFork).

    ``fp8_for``: the nn.Linear that consumes ln(x) in fp8. Under delayed scaling (once
    that layer's amax history exists) the LayerNorm kernel also writes the e4m3 codes
    of its output with the layer's scale and rolls its history, and the codes ride on
    the returned tensor (``_pdt_f8``) for the fp8 GEMM to pick up -- no separate
    quantisation pass over the activation. ``grad_fp8_for``: the fp8 layer whose OUTPUT
    gradient is this fork's input gradient (the residual-stream producer): the LayerNorm
    backward then also writes that layer's e5m2 gradient codes (``_pdt_f8g``)."""
    D = ln.normalized_shape[-1]
    if (len(ln.normalized_shape) != 1 or D not in (256, 512, 768, 1024) or not ln.elementwise_affine
            or x.dtype != torch.bfloat16):
        return x, layer_norm(x, ln)
    meta = None
    if fp8_for is not None and fp8_settings()["scaling"] == "delayed" and D % 128 == 0:
        meta = getattr(fp8_for, "_pdt_fp8_meta", None)
    box: list = []
    if os.environ.get("PDT_FP8_LN_GRAD", "1") == "0":
        grad_fp8_for = None
    only = meta is not None and _ln_codes_only(fp8_for)
    xo, h = _LNFork.apply(x, ln.weight, ln.bias, ln.eps, meta, box, grad_fp8_for, only)
    if box:
        h._pdt_f8 = (box[0][0], box[0][1], fp8_for)
        if only:
            h._pdt_f8_only = True
    return xo, h


def _ln_codes_only(fp8_for) -> bool:
    """The LayerNorm output's bf16 values are not written when its consumer (the fp8 layer
    ``fp8_for``: ViT's qkv / fc1) reads only its e4m3 codes -- an fp8 forward GEMM on the
    codes, and fp8 weight gradients that keep the codes instead of the bf16 input. The
    returned tensor carries ``_pdt_f8_only``; a consumer that would read the values refuses it
    (:func:`_prequant`). PDT_LN_CODES_ONLY=0 writes them anyway."""
    cfg = fp8_settings()
    return (os.environ.get("PDT_LN_CODES_ONLY", "1") == "1" and cfg["dgrad"] and cfg["wgrad"]
            and fp8_for.in_features % 128 == 0 and fp8_for.out_features % 128 == 0)


def _prequant(x, owner):
    """(codes [rows, K], dq) if ``x`` carries fp8 codes made for ``owner`` (ln_fork), else None.
    A codes-only tensor (``_pdt_f8_only``: its bf16 values were never written) may be read by
    ``owner`` alone, and only through an fp8 path that keeps the codes for its weight gradient."""
    pre = getattr(x, "_pdt_f8", None)
    if getattr(x, "_pdt_f8_only", False):
        cfg = fp8_settings()
        if pre is None or pre[2] is not owner or not (cfg["dgrad"] and cfg["wgrad"]):
            raise RuntimeError("this LayerNorm output carries fp8 codes only (its bf16 values were not written) "
                               "and its consumer would read the values: set PDT_LN_CODES_ONLY=0")
    if pre is None or pre[2] is not owner:
        return None
    return pre[0], pre[1]


# =============================================================================
# softmax cross-entropy
# =============================================================================
class _XEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, eps):
        lib = _load()
        logits = logits.contiguous()
        B, V = logits.shape
        is_bf16 = logits.dtype == torch.bfloat16
        if not is_bf16 and logits.dtype != torch.float32:
            logits = logits.float()
        target = target.to(torch.long).contiguous()
        assert target.numel() == B
        lse = torch.empty(B, dtype=torch.float32, device=logits.device)
        rows = torch.empty(B, dtype=torch.float32, device=logits.device)
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        _chk(lib.pdt_xent_fwd(_p(logits), int(is_bf16), _p(target), _p(lse), _p(rows), _p(loss), B, V, float(eps),
                              _s()), "xent_fwd")
        ctx.save_for_backward(logits, target, lse)
        ctx.eps = eps
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, target, lse = ctx.saved_tensors
        B, V = logits.shape
        g = g.float().reshape(1).contiguous()
        dl = torch.empty((B, V), dtype=torch.bfloat16, device=logits.device)
        _chk(_load().pdt_xent_bwd(_p(logits), int(logits.dtype == torch.bfloat16), _p(target), _p(lse), _p(g),
                                  _p(dl), B, V, float(ctx.eps), _s()), "xent_bwd")
        return dl, None, None


def softmax_cross_entropy(logits, target, label_smoothing=0.0):
    if logits.dim() != 2:
        fallback("softmax_cross_entropy", f"logits of shape {tuple(logits.shape)} (kernel: [B, V])")
        return torch.nn.functional.cross_entropy(logits.float(), target, label_smoothing=label_smoothing)
    return _XEnt.apply(logits, target, float(label_smoothing))


# =============================================================================
# ViT ops (torch path for now on GPU as well; native kernels land in ops/vit_ops)
# =============================================================================
def _attn_bwd_q8_target(ctx):
    """(owner, gmeta) when the fp8 attention backward should also write the qkv projection's
    e5m2 gradient codes and bias gradient: delayed scaling with an amax history on the
    projection (``grad_fp8_for`` = the fp8 layer whose output is this attention's only input)
    whose backward is fp8 in both GEMMs. PDT_ATTN_BWD_Q8=0: the separate cast pass."""
    owner = ctx.grad_owner
    if owner is None or os.environ.get("PDT_ATTN_BWD_Q8", "1") != "1":
        return None
    cfg = fp8_settings()
    gmeta = getattr(owner, "_pdt_fp8_gmeta", None)
    if gmeta is None or cfg["scaling"] != "delayed" or not (cfg["dgrad"] and cfg["wgrad"]):
        return None
    return owner, gmeta


class _QKVAttention(torch.autograd.Function):
    """Fused multi-head attention straight off the qkv projection output
    (csrc/attention.hip): qkv [B, T, 3*H*64] -> out [B, T, H*64] (the proj
    GEMM's input layout) with the log-sum-exp saved for the recomputing
    backward, which writes d(qkv) in the qkv layout (the qkv GEMM's dY)."""

    @staticmethod
    def forward(ctx, qkv, H, fp8=False, q8meta=None, box=None, grad_owner=None):
        B, T, D3 = qkv.shape
        assert D3 == 3 * H * 64 and qkv.dtype == torch.bfloat16, "head_dim must be 64, bf16"
        qkv = qkv.contiguous()
        out = torch.empty((B, T, H * 64), dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty((B * H, T), dtype=torch.float32, device=qkv.device)
        scale = 64 ** -0.5
        if fp8 and T <= 256 and q8meta is not None:  # + the projection GEMM's e4m3 input
            codes = torch.empty((B * T, H * 64), dtype=torch.uint8, device=qkv.device)
            part = torch.empty(B * H + 1, dtype=torch.float32, device=qkv.device)
            dq = part[-1:]
            _chk(_load().pdt_attn_fwd_f8_q8(_p(qkv), _p(out), _p(lse), B, T, H, scale, _p(codes), _p(q8meta),
                                            _p(part), _p(dq), _s()), "attn_fwd_f8_q8")
            box.append((codes, dq))
        elif fp8 and T <= 256:  # fp8 QK^T (csrc/attention_f8.hip), fp32 softmax, bf16 PV
            _chk(_load().pdt_attn_fwd_f8(_p(qkv), _p(out), _p(lse), B, T, H, scale, _s()), "attn_fwd_f8")
        elif T <= 256 and os.environ.get("PDT_ATTN_FWD32", "1") == "1":  # 32x32-tile bf16 forward
            _chk(_load().pdt_attn_fwd_tiles(_p(qkv), _p(out), _p(lse), B, T, H, scale, _s()), "attn_fwd_tiles")
        else:
            _chk(_load().pdt_attn_fwd(_p(qkv), _p(out), _p(lse), B, T, H, scale, _s()), "attn_fwd")
        ctx.save_for_backward(qkv, out, lse)
        ctx.H, ctx.scale, ctx.grad_owner, ctx.fp8 = H, scale, grad_owner, bool(fp8)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        B, T, _ = qkv.shape
        dout = dout.to(torch.bfloat16).contiguous()
        delta = torch.empty_like(lse)
        dqkv = torch.empty_like(qkv)
        owner = ctx.grad_owner
        gmeta = getattr(owner, "_pdt_fp8_gmeta", None) if owner is not None else None
        f8bwd = ctx.fp8 and T <= 256 and os.environ.get("PDT_FP8_ATTN_BWD", "1") == "1"
        if not f8bwd and gmeta is not None and T <= 256 and fp8_settings()["scaling"] == "delayed" and \
                os.environ.get("PDT_FP8_ATTN_Q8", "0") == "1":
            # also the e5m2 codes of d(qkv) for the qkv projection's fp8 gradient GEMMs
            codes = torch.empty((B * T, qkv.shape[2]), dtype=torch.uint8, device=qkv.device)
            part = torch.empty(2 * B * ctx.H + 1, dtype=torch.float32, device=qkv.device)
            dq = part[-1:]
            rc = _load().pdt_attn_bwd_q8(_p(qkv), _p(out), _p(dout), _p(lse), _p(delta), _p(dqkv), B, T, ctx.H,
                                         ctx.scale, _p(codes), _p(gmeta), _p(part), _p(dq), _s())
            if rc == 0:
                dqkv._pdt_f8g = (codes, dq, owner)
                return dqkv, None, None, None, None, None
        if f8bwd:
            # fused fp8 backward (csrc/attention_bwd_f8.hip): dQ, dK, dV in one kernel on e4m3 MFMA
            q8 = _attn_bwd_q8_target(ctx)
            if q8 is not None:
                # ... that also writes the qkv projection's e5m2 output gradient (its delayed
                # scale) and bias gradient; the bf16 d(qkv) is then never read (the projection's
                # backward consumes the codes and the bias gradient: _LinearF8), so it is not
                # written unless PDT_ATTN_BWD_Q8_BF16=1
                owner, gmeta = q8
                lib = _load()
                n = qkv.shape[2]
                codes = torch.empty((B * T, n), dtype=torch.uint8, device=qkv.device)
                grid = lib.pdt_attn_bwd_f8_grid(B, ctx.H)
                part = torch.empty(grid + 1, dtype=torch.float32, device=qkv.device)
                dq = part[-1:]
                colpart = torch.empty(B * n + lib.pdt_reduce_rows_work(B, n), dtype=torch.float32,
                                      device=qkv.device)
                db = _grad_buf(getattr(owner, "bias", None), (n,))
                wbf = os.environ.get("PDT_ATTN_BWD_Q8_BF16", "0") == "1"
                _chk(lib.pdt_attn_bwd_f8_q8(_p(qkv), _p(out), _p(dout), _p(lse), _p(dqkv) if wbf else None, B, T,
                                            ctx.H, ctx.scale, _p(codes), _p(gmeta), _p(part), _p(dq), _p(colpart),
                                            _p(db), _s()), "attn_bwd_f8_q8")
                dqkv._pdt_f8g = (codes, dq, owner)
                dqkv._pdt_db = (db, owner)
                if not wbf:
                    dqkv._pdt_f8g_only = owner  # (the values were not written: see _LinearF8)
                return dqkv, None, None, None, None, None
            _chk(_load().pdt_attn_bwd_f8(_p(qkv), _p(out), _p(dout), _p(lse), _p(dqkv), B, T, ctx.H, ctx.scale,
                                         _s()), "attn_bwd_f8")
            return dqkv, None, None, None, None, None
        _chk(_load().pdt_attn_bwd(_p(qkv), _p(out), _p(dout), _p(lse), _p(delta), _p(dqkv), B, T, ctx.H,
                                  ctx.scale, _s()), "attn_bwd")
        return dqkv, None, None, None, None, None


class _ClsAttention(torch.autograd.Function):
    """Attention of token 0's query against all T keys of a packed qkv [B, T, 3*H*64]
    (csrc/attention_cls.hip): the output [B, 1, H*64] and, in backward, the full dqkv (token 0's
    q gradient, every token's k / v gradients, zeros for the other queries)."""

    @staticmethod
    def forward(ctx, qkv, H):
        B, T, D3 = qkv.shape
        qkv = qkv.contiguous()
        if qkv.data_ptr() % 16:  # the kernels read 16-B chunks
            qkv = qkv.clone()
        o = torch.empty((B, 1, D3 // 3), dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(B * H, dtype=torch.float32, device=qkv.device)
        _chk(_load().pdt_cls_attn_fwd(_p(qkv), _p(o), _p(lse), B, T, H, _s()), "cls_attn_fwd")
        ctx.save_for_backward(qkv, o, lse)
        ctx.H = H
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        B, T, _ = qkv.shape
        do = do.to(torch.bfloat16).contiguous()
        if do.data_ptr() % 16:  # the kernel reads 16-B chunks
            do = do.clone()
        dqkv = torch.empty_like(qkv)
        _chk(_load().pdt_cls_attn_bwd(_p(qkv), _p(o), _p(do), _p(lse), _p(dqkv), B, T, ctx.H, _s()), "cls_attn_bwd")
        return dqkv, None


def cls_attention(qkv, num_heads):
    assert qkv.dtype == torch.bfloat16 and qkv.shape[-1] == 3 * 64 * num_heads and qkv.shape[1] <= 256
    return _ClsAttention.apply(qkv, num_heads)


def qkv_attention(qkv, num_heads, fp8=False, fp8_for=None, grad_fp8_for=None):
    """softmax(q k^T / 8) v over heads of 64 for a packed [B, T, 3*H*64] qkv. ``fp8``: the
    score GEMM on e4m3 MFMA (per-head / per-tile power-of-two scales, T <= 256) and the
    fused fp8 backward (csrc/attention_bwd_f8.hip; PDT_FP8_ATTN_BWD=0: the bf16 one). ``fp8_for``: the fp8 layer consuming
    the output (the attention projection): under delayed scaling the kernel also writes
    its e4m3 input (``_pdt_f8`` on the result, as :func:`ln_fork` does); ``grad_fp8_for``:
    the fp8 layer that produced qkv -- the backward then also writes its e5m2 output
    gradient (``_pdt_f8g`` on d(qkv))."""
    meta = None
    # Default "fwd": the fp8 attention forward also writes the projection's e4m3 input codes
    # (same-box A/B, round 6 q29: 11 626 / 11 640 vs 11 546 / 11 558 img/s with the separate cast
    # pass, "0"). "1" adds the bf16 backward's d(qkv) codes (the fp8 backward writes its own:
    # _attn_bwd_q8_target); in round 4 (r4e-r4h) the then-kernels' uncoalesced code stores cost
    # more than the casts (6.32k vs 6.40k img/s), which is why this was off until round 6.
    q8 = os.environ.get("PDT_FP8_ATTN_Q8", "fwd")
    if q8 != "1":
        if not fp8:  # (the fp8 backward's epilogue writes the gradient codes: _attn_bwd_q8_target)
            grad_fp8_for = None
        if q8 != "fwd":
            fp8_for = None
    if fp8 and fp8_for is not None and fp8_settings()["scaling"] == "delayed":
        meta = getattr(fp8_for, "_pdt_fp8_meta", None)
    box: list = []
    out = _QKVAttention.apply(qkv, num_heads, bool(fp8), meta, box, grad_fp8_for if fp8 else None)
    if box:
        out._pdt_f8 = (box[0][0], box[0][1], fp8_for)
    return out


def attention(q, k, v):
    """softmax(q k^T / sqrt(64)) v for [B, H, T, 64] q / k / v on the fused attention
    kernel (packs them into the [B, T, 3*H*64] layout :func:`qkv_attention` reads)."""
    B, H, T, d = q.shape
    if d != 64 or k.shape != q.shape or v.shape != q.shape or q.dtype != torch.bfloat16:
        fallback("attention", f"q {tuple(q.shape)} {q.dtype} (kernel: head dim 64, bf16, self-attention shapes)")
        return torch.nn.functional.scaled_dot_product_attention(q, k, v)
    qkv = torch.stack([q, k, v], dim=2).permute(0, 3, 2, 1, 4).reshape(B, T, 3 * H * d)
    return qkv_attention(qkv, H).view(B, T, H, d).transpose(1, 2)


class _PatchEmbed(torch.autograd.Function):
    """Non-overlapping patch conv as an implicit GEMM whose NHWC output IS the
    [B, N_patches, D] token matrix (no transpose pass)."""

    @staticmethod
    def forward(ctx, x, w, b, conv):
        N, C, H, W = x.shape
        Cs = C if C % 8 == 0 else 8
        x = x.to(torch.bfloat16)
        if Cs != C:
            x = torch.nn.functional.pad(_cl(x).permute(0, 2, 3, 1), (0, Cs - C)).permute(0, 3, 1, 2)
        x = _cl(x)
        Cout = w.shape[0]
        g = _fwd_geom(N, H, W, Cs, conv)
        wb = bf16_weight(w, pad_cin_to=Cs if Cs != C else None)
        y = _empty_cl(N, Cout, g["Ho"], g["Wo"], torch.bfloat16, x.device)
        conv_nt(x, wb, y, bias=b.float().contiguous() if b is not None else None,
                **_fwd_nt_geom(N, H, W, Cs, Cout, g))
        u = _Unit()
        u.x, u.w, u.N, u.C, u.Cs, u.H, u.W, u.Cout, u.g = x, w, N, C, Cs, H, W, Cout, g
        ctx.u = u
        ctx.has_b = b is not None
        return y.permute(0, 2, 3, 1).reshape(N, g["Ho"] * g["Wo"], Cout)

    @staticmethod
    def backward(ctx, dtok):
        u = ctx.u
        N, Cout = u.N, u.Cout
        dy = dtok.to(torch.bfloat16).reshape(N, u.g["Ho"], u.g["Wo"], Cout).permute(0, 3, 1, 2)
        dy = _cl(dy)
        dw = _unit_dw(dy, u) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = colsum(dy, N * u.g["Ho"] * u.g["Wo"], Cout)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _unit_dx(dy, u)
        del ctx.u
        return dx, dw, db, None


class _PatchLinear(torch.autograd.Function):
    """Non-overlapping patch conv as patchify + plain GEMM: one strided copy forms the
    [B*N_patches, C*KH*KW] patch matrix (bf16, in the weight's own element order), then the
    bf16 GEMM (bias in its epilogue) writes the token matrix and the weight gradient + bias
    sums are one plain wgrad call on the same patch matrix. For 3-channel images this is
    K = 768 instead of the implicit GEMM's channel-padded K = 2048 (ViT-B/16), and no pad pass.
    The reference runs torch's conv (torchvision vit_b_16 ``conv_proj``)."""

    @staticmethod
    def forward(ctx, x, w, b, conv):
        N, C, H, W = x.shape
        Cout, _, KH, KW = w.shape
        nh, nw = H // KH, W // KW
        K = C * KH * KW
        kkc = w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous()
        xv = x.view(N, C, nh, KH, nw, KW)
        pm = torch.empty((N * nh * nw, K), dtype=torch.bfloat16, device=x.device)
        if kkc:  # weight memory order (kh, kw, c)
            pm.view(N, nh, nw, KH, KW, C).copy_(xv.permute(0, 2, 4, 3, 5, 1))
            wb = bf16_weight(w).permute(0, 2, 3, 1).reshape(Cout, K)
        else:    # (c, kh, kw)
            pm.view(N, nh, nw, C, KH, KW).copy_(xv.permute(0, 2, 4, 1, 3, 5))
            wb = w.detach().reshape(Cout, K).to(torch.bfloat16).contiguous()
        y = torch.empty((N * nh * nw, Cout), dtype=torch.bfloat16, device=x.device)
        _gemm_bf16(pm, wb, y, bias=b.float().contiguous() if b is not None else None)
        ctx.save_for_backward(pm)
        ctx.meta = (w, b, kkc, N, nh * nw)
        return y.view(N, nh * nw, Cout)

    @staticmethod
    def backward(ctx, dtok):
        (pm,) = ctx.saved_tensors
        w, b, kkc, N, npatch = ctx.meta
        Cout = w.shape[0]
        K = pm.shape[1]
        want_dw, want_db = ctx.needs_input_grad[1], b is not None and ctx.needs_input_grad[2]
        dy2 = dtok.reshape(-1, Cout).to(torch.bfloat16).contiguous()
        dw = db = None
        if want_dw:
            if kkc:
                dw = _grad_buf(w, tuple(w.shape), torch.channels_last)
                dw2 = dw.permute(0, 2, 3, 1).reshape(Cout, K)
            else:
                dw = _grad_buf(w, tuple(w.shape))
                dw2 = dw.view(Cout, K)
            db = _grad_buf(b, (Cout,)) if want_db else None
            conv_wgrad(dy2, pm, dw2, M=dy2.shape[0], Mo=Cout, No=K, ldy=Cout, Hs=1, Ws=1, C=K, Hm=1, Wm=1, sh=1,
                       sw=1, oh0=0, ow0=0, dh=1, dw=1, ntw=1, bias_out=db)
            dw = dw.to(w.dtype) if dw.dtype != w.dtype else dw
        elif want_db:
            db = colsum(dy2, dy2.shape[0], Cout)
        return None, dw, db, None


class _EmbedTokens(torch.autograd.Function):
    """x[:, 0] = cls + pos[0], x[:, 1:] = tok + pos[1:] written straight into the [B, N+1, D]
    buffer (one pass over the tokens instead of torch.cat then the broadcast add). Backward:
    d_pos = sum over the batch, d_cls = d_pos[0] (cls and pos[0] add to the same token of every
    image), d_tok a view of the incoming gradient. The reference gets its token assembly from
    torchvision's vit_b_16 (class token concat + pos-embedding add)."""

    @staticmethod
    def forward(ctx, tok, cls_token, pos_embed):
        B, N, D = tok.shape
        x = torch.empty((B, N + 1, D), dtype=tok.dtype, device=tok.device)
        pos = pos_embed.detach().to(tok.dtype).reshape(N + 1, D)
        torch.add(tok, pos[1:], out=x[:, 1:])
        x[:, 0] = (cls_token.detach().reshape(D) + pos_embed.detach().reshape(N + 1, D)[0]).to(tok.dtype)
        ctx.meta = (cls_token.shape, cls_token.dtype, pos_embed.shape, pos_embed.dtype)
        return x

    @staticmethod
    def backward(ctx, dx):
        cshape, cdtype, pshape, pdtype = ctx.meta
        need_pos = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        dpos = dx.sum(0, dtype=torch.float32) if need_pos else None
        dcls = dpos[0].reshape(cshape).to(cdtype) if ctx.needs_input_grad[1] else None
        dp = dpos.reshape(pshape).to(pdtype) if ctx.needs_input_grad[2] else None
        dtok = dx[:, 1:] if ctx.needs_input_grad[0] else None
        return dtok, dcls, dp


def embed_tokens(tok, cls_token, pos_embed):
    B, N, D = tok.shape
    if os.environ.get("PDT_EMBED_FUSED", "1") != "1":  # A/B switch: torch.cat + add
        return torch.cat([cls_token.to(tok.dtype).expand(B, -1, -1), tok], dim=1) + pos_embed.to(tok.dtype)
    if cls_token.numel() != D or pos_embed.numel() != (N + 1) * D:
        fallback("embed_tokens", f"cls {tuple(cls_token.shape)} pos {tuple(pos_embed.shape)} for tokens {tuple(tok.shape)}")
        return torch.cat([cls_token.to(tok.dtype).expand(B, -1, -1), tok], dim=1) + pos_embed.to(tok.dtype)
    return _EmbedTokens.apply(tok, cls_token, pos_embed)


def _patch_linear_ok(x, conv) -> bool:
    if os.environ.get("PDT_PATCH_LINEAR", "1") != "1" or x.requires_grad:
        return False
    K = conv.in_channels * conv.kernel_size[0] * conv.kernel_size[1]
    return K % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32)


def patch_embed(x, conv):
    KH, KW = conv.kernel_size
    if (conv.stride != conv.kernel_size or conv.padding != (0, 0) or conv.out_channels % 8 or conv.groups != 1
            or conv.dilation != (1, 1) or x.dim() != 4 or x.shape[2] % KH or x.shape[3] % KW
            or (x.shape[1] % 8 and x.shape[1] > 8)):
        fallback("patch_embed", f"conv {tuple(conv.kernel_size)}/{tuple(conv.stride)} on {tuple(x.shape)} "
                                "(kernel: non-overlapping patches, bias-any, channels <= 8 or % 8 == 0)")
        y = conv(x)
        return y.flatten(2).transpose(1, 2)
    if _patch_linear_ok(x, conv):
        return _PatchLinear.apply(x, conv.weight, conv.bias, conv)
    return _PatchEmbed.apply(x, conv.weight, conv.bias, conv)


# =============================================================================
# MnistModel (the reference's LeNet, /root/reference/model/model.py:6-22) as two
# whole-network kernels (csrc/lenet.hip: one workgroup per image, all layers in
# LDS, fp32 like the reference), and the NLL loss (/root/reference/model/loss.py:5).
# =============================================================================
def lenet_supported(model, x) -> bool:
    c1, c2, f1, f2 = model.conv1, model.conv2, model.fc1, model.fc2
    return (x.is_cuda and x.dim() == 4 and tuple(x.shape[1:]) == (1, 28, 28)
            and (c1.in_channels, c1.out_channels, c1.kernel_size, c1.stride, c1.padding) == (1, 10, (5, 5), (1, 1), (0, 0))
            and (c2.in_channels, c2.out_channels, c2.kernel_size, c2.stride, c2.padding) == (10, 20, (5, 5), (1, 1), (0, 0))
            and (f1.in_features, f1.out_features) == (320, 50) and f2.in_features == 50 and f2.out_features <= 64
            and all(t is not None for t in (c1.bias, c2.bias, f1.bias, f2.bias)))


def _lenet_params(model):
    return [t.detach().float().contiguous() for t in (model.conv1.weight, model.conv1.bias, model.conv2.weight,
                                                      model.conv2.bias, model.fc1.weight, model.fc1.bias,
                                                      model.fc2.weight, model.fc2.bias)]


class _LeNet(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, wf1, bf1, wf2, bf2, training, p2, p1, seed, masks):
        x = x.float().contiguous()
        ps = [t.float().contiguous() for t in (w1, b1, w2, b2, wf1, bf1, wf2, bf2)]
        B, NC = x.shape[0], wf2.shape[0]
        logp = torch.empty((B, NC), dtype=torch.float32, device=x.device)
        m2, m1 = (masks if masks is not None else (None, None))
        _chk(_load().pdt_lenet_fwd(*[_p(t) for t in [x] + ps], B, NC, int(training), float(p2), float(p1),
                                   seed & 0xFFFFFFFF, _p(logp), _p(m2), _p(m1), _s()), "lenet_fwd")
        ctx.save_for_backward(x, *ps)
        ctx.meta = (B, NC, int(training), float(p2), float(p1), seed & 0xFFFFFFFF)
        return logp

    @staticmethod
    def backward(ctx, g):
        x, *ps = ctx.saved_tensors
        B, NC, training, p2, p1, seed = ctx.meta
        lib = _load()
        row = lib.pdt_lenet_grad_row(NC)
        part = torch.empty(B * row, dtype=torch.float32, device=x.device)
        flat = torch.empty(row, dtype=torch.float32, device=x.device)
        g = g.float().contiguous()
        _chk(lib.pdt_lenet_bwd(*[_p(t) for t in [x] + ps], B, NC, training, p2, p1, seed, _p(g), _p(part), _p(flat),
                               _s()), "lenet_bwd")
        grads, off = [], 0
        for t in ps:  # flat layout = parameter order (csrc/lenet.hip O_*)
            grads.append(flat[off:off + t.numel()].view(t.shape))
            off += t.numel()
        assert off == row
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("native LeNet does not produce an input gradient")
        return (None, *grads, None, None, None, None, None)


def lenet_forward(model, x, masks=None, seed=None):
    """log-probabilities of MnistModel on x [B, 1, 28, 28] (Dropout2d / dropout active in training)."""
    p2 = model.conv2_drop.p if model.training else 0.0
    p1 = 0.5 if model.training else 0.0
    if seed is None:
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if model.training else 0  # host RNG: no device sync
    return _LeNet.apply(x, model.conv1.weight, model.conv1.bias, model.conv2.weight, model.conv2.bias,
                        model.fc1.weight, model.fc1.bias, model.fc2.weight, model.fc2.bias, model.training, p2, p1,
                        seed, masks)


class _TargetCheck:
    """Lazy device-side check of NLL targets: each forward's count of out-of-range
    targets is copied (non-blocking) to pinned host memory; the NEXT call reads it once
    its event has completed and raises -- no host sync inside the step. The loss of
    the offending batch itself is already NaN (csrc/lenet.hip nll_fwd_kernel).
    ``PDT_CHECK_TARGETS=sync`` checks every call synchronously instead."""

    def __init__(self):
        self.pending = []  # (event, pinned host tensor)

    def record(self, bad: torch.Tensor):
        if _capturing():  # inside a HIP-graph capture: no host copies / events (the NaN loss remains)
            return
        if os.environ.get("PDT_CHECK_TARGETS", "lazy") == "sync":
            n = float(bad.item())
            if n:
                raise ValueError(f"nll_loss: {int(n)} target(s) out of range [0, num_classes)")
            return
        host = torch.empty(1, dtype=torch.float32, pin_memory=True)
        host.copy_(bad.reshape(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((ev, host))

    MAX_PENDING = 64  # beyond this the oldest check is waited for (never dropped)

    def poll(self, block=False):
        """Raise if any finished check saw an out-of-range target. ``block``: wait for every
        pending check (end of an epoch / run: the last batches' checks are read too). Every
        check is kept until it has been read; when more than MAX_PENDING are queued the
        oldest is waited for instead of dropped."""
        if _capturing():
            return
        keep = []
        for i, (ev, host) in enumerate(self.pending):
            if not (block or len(self.pending) - i > self.MAX_PENDING) and not ev.query():
                keep.append((ev, host))
                continue
            ev.synchronize()
            if float(host[0]):
                self.pending = []
                raise ValueError(f"nll_loss: {int(host[0])} target(s) out of range [0, num_classes) "
                                 "in an earlier batch (its loss was NaN)")
        self.pending = keep


def check_targets_pending():
    """Read every outstanding NLL target check (blocking); raises on an out-of-range target.
    The Trainer calls it at the end of each epoch."""
    _TARGETS.poll(block=True)


_TARGETS = _TargetCheck()


class _NLL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logp, target, ignore_index):
        _TARGETS.poll()
        logp = logp.float().contiguous()
        target = target.to(torch.long).contiguous()
        B, C = logp.shape
        assert target.numel() == B
        out = torch.empty(3, dtype=torch.float32, device=logp.device)  # loss, count, #out-of-range targets
        _chk(_load().pdt_nll_fwd(_p(logp), _p(target), B, C, int(ignore_index), _p(out[0]), _p(out[1]),
                                 _p(out[2]), _s()), "nll_fwd")
        _TARGETS.record(out[2])
        ctx.save_for_backward(target, out)
        ctx.meta = (B, C, int(ignore_index))
        return out[0].clone()

    @staticmethod
    def backward(ctx, g):
        target, out = ctx.saved_tensors
        B, C, ignore = ctx.meta
        d = torch.empty((B, C), dtype=torch.float32, device=target.device)
        _chk(_load().pdt_nll_bwd(_p(target), _p(g.float().reshape(1).contiguous()), _p(out[1]), B, C, ignore, _p(d),
                                 _s()), "nll_bwd")
        return d, None, None


def nll_loss(logp, target, ignore_index=-100):
    return _NLL.apply(logp, target, ignore_index)

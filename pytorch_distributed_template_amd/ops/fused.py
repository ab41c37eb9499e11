"""Fused op entry points used by the models.

Each function has two implementations:
  * ``native``: hand-written HIP/CDNA4 kernels (``csrc/*.hip``) wrapped in
    ``torch.autograd.Function``s (see ``ops/native_ops.py``);
  * ``torch``: plain PyTorch ops -- used on CPU (gloo plumbing tests), as the
    fp32 reference in numerics tests, and as the "stock ROCm stack" baseline
    in ``bench.py --backend torch``.

The backend is chosen per process with :func:`set_backend` (default:
``native`` for GPU tensors when the extension is built, ``torch`` on CPU).
The reference has no fused ops at all -- it runs stock cuDNN/cuBLAS kernels
(SURVEY.md §2.6(a)).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

_BACKEND = os.environ.get("PDT_BACKEND", "auto")  # auto | native | torch


def set_backend(name: str) -> None:
    global _BACKEND
    assert name in ("auto", "native", "torch"), name
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


def use_native(x: torch.Tensor) -> bool:
    """True when ``x``'s op should run on the native HIP kernels (GPU tensor,
    backend not ``torch``, library present -- ``native`` raises if it is missing)."""
    return _use_native(x)


def _use_native(x: torch.Tensor) -> bool:
    if _BACKEND == "torch" or not x.is_cuda:
        return False
    from . import native_ops  # noqa: WPS433 (lazy: avoids loading the .so on CPU)
    if _BACKEND == "native":
        native_ops.require()
        return True
    return native_ops.available()


# ----------------------------------------------------------------------------
# reference (torch) implementations
# ----------------------------------------------------------------------------
def _torch_conv_bn_act(x, conv: nn.Conv2d, bn: nn.BatchNorm2d, residual=None, relu=True):
    # plain ops; under torch.autocast(bf16) conv runs in bf16 and BN keeps fp32 params
    y = conv(x)
    y = bn(y)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y)
    return y


def conv_bn_act(x, conv: nn.Conv2d, bn: nn.BatchNorm2d, residual=None, relu: bool = True):
    """y = act(BN(conv(x)) [+ residual]) with training-mode batch statistics."""
    if _use_native(x):
        from . import native_ops
        return native_ops.conv_bn_act(x, conv, bn, residual, relu)
    return _torch_conv_bn_act(x, conv, bn, residual, relu)


def bottleneck(x, blk):
    """ResNet bottleneck block; the native path runs it as one fused autograd node."""
    if _use_native(x):
        from . import native_ops
        out = native_ops.bottleneck(x, blk)
        if out is not None:
            return out
    if blk.downsample is not None:
        identity = conv_bn_act(x, blk.downsample[0], blk.downsample[1], relu=False)
    else:
        identity = x
    out = conv_bn_act(x, blk.conv1, blk.bn1, relu=True)
    out = conv_bn_act(out, blk.conv2, blk.bn2, relu=True)
    return conv_bn_act(out, blk.conv3, blk.bn3, residual=identity, relu=True)


def bottleneck_chain(x, blocks):
    """A sequence of bottleneck blocks. Native: each block's final BN(+res)+ReLU pass is
    folded into the next block's first 1x1 GEMM (``native_ops.bottleneck_chain``)."""
    blocks = list(blocks)
    if _use_native(x):
        from . import native_ops
        x, n = native_ops.bottleneck_chain(x, blocks)
        blocks = blocks[n:]
    for blk in blocks:
        x = bottleneck(x, blk)
    return x


def conv_bn_relu_maxpool(x, conv: nn.Conv2d, bn: nn.BatchNorm2d, kernel_size=3, stride=2, padding=1):
    """max_pool2d(relu(BN(conv(x)))) -- the ResNet stem. Native: one node whose
    max-pool applies the BN affine + ReLU on the fly (no full-resolution activation)."""
    if _use_native(x):
        from . import native_ops
        out = native_ops.stem_pool(x, conv, bn, kernel_size, stride, padding)
        if out is not None:
            return out
    return max_pool2d(conv_bn_act(x, conv, bn, relu=True), kernel_size, stride, padding)


def max_pool2d(x, kernel_size=3, stride=2, padding=1):
    if _use_native(x):
        from . import native_ops
        return native_ops.max_pool2d(x, kernel_size, stride, padding)
    return F.max_pool2d(x, kernel_size, stride, padding)


def global_avg_pool(x):
    """[N,C,H,W] (any memory format) -> [N,C]."""
    if _use_native(x):
        from . import native_ops
        return native_ops.global_avg_pool(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def _torch_linear(x, fc: nn.Linear, act=None):
    if x.dtype != fc.weight.dtype and not torch.is_autocast_enabled(x.device.type):
        x = x.to(fc.weight.dtype)
    y = fc(x)
    if act == "gelu":
        y = F.gelu(y, approximate="tanh")
    elif act == "relu":
        y = F.relu(y)
    return y


def linear(x, fc: nn.Linear, act: str | None = None, fp8: bool = False, residual=None):
    """y = act(x @ W^T + b) (+ residual). ``act`` in {None, "gelu", "relu"}; ``fp8`` selects
    the e4m3 GEMM with per-tensor scaling on the native path (ignored on torch path).
    Native: the residual add runs in the GEMM epilogue."""
    if _use_native(x):
        from . import native_ops
        return native_ops.linear(x, fc, act=act, fp8=fp8, residual=residual)
    y = _torch_linear(x, fc, act)
    return y if residual is None else y + residual


def mlp(x, m: nn.Module, fp8: bool = False, residual=None):
    """fc2(gelu_tanh(fc1(x))) (+ residual) of a transformer MLP with ``fc1`` / ``fc2``.
    Native: one autograd node (GELU backward fused into fc2's data-gradient GEMM,
    bias gradients from the weight-gradient kernels, residual in fc2's epilogue)."""
    if _use_native(x):
        from . import native_ops
        return native_ops.mlp(x, m, fp8=fp8, residual=residual)
    y = _torch_linear(_torch_linear(x, m.fc1, "gelu"), m.fc2)
    return y if residual is None else y + residual


def layer_norm(x, ln: nn.LayerNorm):
    if _use_native(x):
        from . import native_ops
        return native_ops.layer_norm(x, ln)
    return ln(x)


def ln_fork(x, ln: nn.LayerNorm, fp8_for: nn.Linear | None = None, grad_fp8_for: nn.Linear | None = None):
    """(x, ln(x)) for a pre-norm residual block. Native: the residual gradient of x
    and the normalised branch's gradient are summed inside LayerNorm's backward;
    ``fp8_for`` (the fp8 layer consuming ln(x)) lets the LayerNorm kernel emit that
    layer's e4m3 input directly, and ``grad_fp8_for`` (the fp8 layer that produced x) its
    e5m2 output gradient in the backward."""
    if _use_native(x):
        from . import native_ops
        return native_ops.ln_fork(x, ln, fp8_for, grad_fp8_for)
    return x, ln(x)


def ln_add_fork(y, r, ln: nn.LayerNorm, fp8_for: nn.Linear | None = None, grad_fp8_for: nn.Linear | None = None):
    """(y + r, ln(y + r)): :func:`ln_fork` with the block's residual add done by the native
    LayerNorm kernel (it reads y and r and writes the sum) instead of the producing GEMM's
    epilogue."""
    if _use_native(y):
        from . import native_ops
        return native_ops.ln_add_fork(y, r, ln, fp8_for, grad_fp8_for)
    s = y + r
    return s, ln(s)


def attention(q, k, v):
    """softmax(q k^T / sqrt(d)) v for [B,H,T,d] tensors (non-causal)."""
    if _use_native(q):
        from . import native_ops
        return native_ops.attention(q, k, v)
    return F.scaled_dot_product_attention(q, k, v)


def qkv_attention(qkv, num_heads: int, fp8: bool = False, fp8_for: nn.Linear | None = None,
                  grad_fp8_for: nn.Linear | None = None):
    """Multi-head attention on a packed qkv projection [B, T, 3*H*hd] -> [B, T, H*hd].
    Native path: one fused MFMA kernel (hd = 64; ``fp8``: e4m3 score GEMM); torch path: SDPA."""
    B, T, D3 = qkv.shape
    hd = D3 // (3 * num_heads)
    if _use_native(qkv):
        from . import native_ops
        if hd == 64 and qkv.dtype == torch.bfloat16:
            return native_ops.qkv_attention(qkv, num_heads, fp8=fp8, fp8_for=fp8_for, grad_fp8_for=grad_fp8_for)
        native_ops.fallback("qkv_attention", f"head dim {hd}, {qkv.dtype} (kernel: head dim 64, bf16)")
    q, k, v = qkv.view(B, T, 3, num_heads, hd).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(q, k, v)
    return o.transpose(1, 2).reshape(B, T, num_heads * hd)


def cls_attention(qkv, num_heads: int):
    """Attention of token 0's query only (against every key / value) on a packed qkv
    [B, T, 3*H*hd] -> [B, 1, H*hd]: what a classifier that reads token 0 needs from the last
    block. Native path: one small kernel per direction (hd = 64, T <= 256); torch path: the
    same math in fp32."""
    B, T, D3 = qkv.shape
    hd = D3 // (3 * num_heads)
    if _use_native(qkv):
        from . import native_ops
        if hd == 64 and qkv.dtype == torch.bfloat16 and T <= 256:
            return native_ops.cls_attention(qkv, num_heads)
        native_ops.fallback("cls_attention", f"head dim {hd}, {qkv.dtype}, T {T} (kernel: 64, bf16, T <= 256)")
    q, k, v = qkv.view(B, T, 3, num_heads, hd).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(q[:, :, :1], k, v)
    return o.transpose(1, 2).reshape(B, 1, num_heads * hd)


def patch_embed(x, conv: nn.Conv2d):
    """Non-overlapping patch conv -> [B, N, D] tokens."""
    if _use_native(x):
        from . import native_ops
        return native_ops.patch_embed(x, conv)
    y = conv(x)
    return y.flatten(2).transpose(1, 2)


def embed_tokens(tok, cls_token, pos_embed):
    """[cls; tok] + pos for [B, N, D] patch tokens -> [B, N+1, D]. Native path: one pass
    writing the token buffer (no concatenated intermediate); torch path: cat + add."""
    if _use_native(tok):
        from . import native_ops
        return native_ops.embed_tokens(tok, cls_token, pos_embed)
    cls = cls_token.to(tok.dtype).expand(tok.shape[0], -1, -1)
    return torch.cat([cls, tok], dim=1) + pos_embed.to(tok.dtype)


def softmax_cross_entropy(logits, target, label_smoothing: float = 0.0):
    """Mean softmax cross-entropy (fused fwd/bwd kernel on the native path)."""
    if _use_native(logits):
        from . import native_ops
        return native_ops.softmax_cross_entropy(logits, target, label_smoothing)
    return F.cross_entropy(logits.float(), target, label_smoothing=label_smoothing)

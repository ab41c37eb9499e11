"""ViT-B/16 (image 224, patch 16, d=768, 12 heads, MLP 3072, depth 12).

Not present in the reference; BASELINE.json config #5 ("ViT-B/16 fp8
synthetic 3x224x224") defines it. Shapes per SURVEY §2.6(b).

The model is written against ``ops.fused`` entry points so the native HIP
path (LayerNorm, bias+GELU epilogue, fused attention, and fp8 GEMMs with
per-tensor amax scaling when ``fp8=True``) and the torch reference path share
one module tree. Parameter names follow the common ``patch_embed / cls_token /
pos_embed / blocks.N.{norm1,attn.qkv,attn.proj,norm2,mlp.fc1,mlp.fc2} / norm /
head`` scheme.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..base.base_model import BaseModel
from ..ops import fused


def _fp8_attn() -> bool:
    """fp8 score GEMM in attention for fp8 models (PDT_FP8_ATTN=0 keeps it bf16)."""
    import os
    return os.environ.get("PDT_FP8_ATTN", "1") == "1"


def _cls_prune(x, setting) -> bool:
    """Whether the last block computes the class token's row only (see Block.forward).
    ``setting`` None: on the native kernel path (the stock torch path stays the plain model, as
    the reference-equivalent baseline); PDT_VIT_CLS_PRUNE=0/1 overrides."""
    import os
    env = os.environ.get("PDT_VIT_CLS_PRUNE")
    if env is not None:
        return env == "1"
    return fused.use_native(x) if setting is None else bool(setting)


def _ln_add() -> bool:
    """fp8 models: the blocks' residual adds in the next LayerNorm kernel instead of the proj /
    fc2 GEMM epilogues (PDT_LN_ADD=0 keeps them in the epilogues)."""
    import os
    return os.environ.get("PDT_LN_ADD", "1") == "1"


class Attention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.qkv = nn.Linear(dim, dim * 3)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x, fp8=False, residual=None):
        qkv = fused.linear(x, self.qkv, fp8=fp8)                          # [B,T,3D]
        # (fp8: the attention kernels also write the projection GEMM's e4m3 input and, in
        # backward, the qkv projection's e5m2 output gradient)
        o = fused.qkv_attention(qkv, self.num_heads, fp8=fp8 and _fp8_attn(),
                                fp8_for=self.proj if fp8 else None,
                                grad_fp8_for=self.qkv if fp8 else None)  # [B,T,D]
        return fused.linear(o, self.proj, fp8=fp8, residual=residual)     # (+ residual in the epilogue)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x, fp8=False, residual=None):
        return fused.mlp(x, self, fp8=fp8, residual=residual)


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x, fp8=False, prev_fc2=None, pending=None, defer=False, cls_only=False):
        # pre-norm residual block; the residual adds ride the proj / fc2 GEMM epilogues and
        # their gradients are summed inside the LayerNorm backward (fused.ln_fork)
        # (fp8: the LayerNorm forward kernels also write the e4m3 inputs of qkv / fc1, and
        # the LayerNorm backward kernels the e5m2 output gradients of the previous block's
        # fc2 / this block's proj -- the layers that produced their inputs).
        # fp8 with _ln_add(): the adds move into the next LayerNorm kernel (fused.ln_add_fork)
        # so proj / fc2 are plain GEMMs (no addend epilogue); ``pending`` = the
        # previous block's (fc2 output, residual) pair, ``defer``: return this block's pair.
        if pending is not None:
            x, h = fused.ln_add_fork(pending[0], pending[1], self.norm1, self.attn.qkv if fp8 else None,
                                     prev_fc2 if fp8 else None)
        else:
            x, h = fused.ln_fork(x, self.norm1, self.attn.qkv if fp8 else None, prev_fc2 if fp8 else None)
        if cls_only:
            return self._forward_cls(x, h, fp8)
        if fp8 and _ln_add():
            y = self.attn(h, fp8=fp8)
            x, h = fused.ln_add_fork(y, x, self.norm2, self.mlp.fc1, self.attn.proj)
        else:
            x = self.attn(h, fp8=fp8, residual=x)
            x, h = fused.ln_fork(x, self.norm2, self.mlp.fc1 if fp8 else None, self.attn.proj if fp8 else None)
        if defer:
            return self.mlp(h, fp8=fp8), x
        return self.mlp(h, fp8=fp8, residual=x)

    def _forward_cls(self, x, h, fp8):
        """The block for a consumer that reads token 0 only (the classifier after the LAST
        block): keys and values of every token (qkv over all rows), but the attention output,
        projection, residual, LayerNorm 2 and MLP of the class token's row alone -> [B, 1, D].
        The model's output and every parameter gradient are those of the full block (the other
        196 output rows feed nothing); it removes ~1/12 of the proj + MLP GEMM work and the
        block's element passes over the other rows."""
        qkv = fused.linear(h, self.attn.qkv, fp8=fp8)
        o = fused.cls_attention(qkv, self.attn.num_heads)          # [B, 1, D]
        x0 = x[:, :1].contiguous()
        if fp8 and _ln_add():
            y = fused.linear(o, self.attn.proj, fp8=fp8)
            x0, h0 = fused.ln_add_fork(y, x0, self.norm2, self.mlp.fc1, self.attn.proj)
        else:
            x0 = fused.linear(o, self.attn.proj, fp8=fp8, residual=x0)
            x0, h0 = fused.ln_fork(x0, self.norm2, self.mlp.fc1 if fp8 else None, self.attn.proj if fp8 else None)
        return self.mlp(h0, fp8=fp8, residual=x0)


class VisionTransformer(BaseModel):
    def __init__(self, image_size=224, patch_size=16, in_chans=3, num_classes=1000, embed_dim=768,
                 depth=12, num_heads=12, mlp_ratio=4.0, fp8=False, cls_prune=None):
        super().__init__()
        self.patch_size = patch_size
        self.fp8 = fp8
        self.cls_prune = cls_prune  # None: on the native path (_cls_prune)
        self.patch_embed = nn.Conv2d(in_chans, embed_dim, patch_size, stride=patch_size)
        n_patches = (image_size // patch_size) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, n_patches + 1, embed_dim))
        self.blocks = nn.ModuleList([Block(embed_dim, num_heads, mlp_ratio) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)
        self.head = nn.Linear(embed_dim, num_classes)
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.trunc_normal_(self.cls_token, std=0.02)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)
        fan_in = in_chans * patch_size * patch_size
        nn.init.trunc_normal_(self.patch_embed.weight, std=math.sqrt(1.0 / fan_in))

    def forward(self, x):
        x = fused.patch_embed(x, self.patch_embed)                 # [B, N, D]
        x = fused.embed_tokens(x, self.cls_token, self.pos_embed)  # [B, N+1, D]
        prev = None
        pending = None
        defer = self.fp8 and _ln_add()
        prune = _cls_prune(x, self.cls_prune)
        for i, blk in enumerate(self.blocks):
            last = i == len(self.blocks) - 1
            out = blk(x, fp8=self.fp8, prev_fc2=prev, pending=pending, defer=defer and not last,
                      cls_only=prune and last)
            if defer and not last:
                pending, x = out, None
            else:
                x, pending = out, None
            prev = blk.mlp.fc2
        x = fused.layer_norm(x[:, 0], self.norm)
        return fused.linear(x, self.head)


def vit_b_16(num_classes=1000, **kw):
    return VisionTransformer(num_classes=num_classes, **kw)


class ViT_B_16(VisionTransformer):
    def __init__(self, num_classes=1000, fp8=False, **kw):
        super().__init__(num_classes=num_classes, fp8=fp8, **kw)

"""fp8 attention (e4m3 score GEMM, csrc/attention_f8.hip) is on by default for fp8 ViTs;
its forward differs from exact attention by ~6 % (tests/test_vit_fusion_gpu.py budget).
This pins what matters for training: on a fixed seed, a small fp8 ViT trained with fp8
attention follows the loss curve of the same model with bf16 attention.

Task: memorise 256 synthetic 64x64 images with random labels (a learnable, fixed
dataset) with AdamW; 150 steps each arm, identical init, data order and fp8 GEMMs."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from pytorch_distributed_template_amd.models.vit import VisionTransformer  # noqa: E402
from pytorch_distributed_template_amd.ops import fused  # noqa: E402
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402
from pytorch_distributed_template_amd.optim import FusedAdamW  # noqa: E402


def _train(fp8_attn: bool, steps=150):
    os.environ["PDT_FP8_ATTN"] = "1" if fp8_attn else "0"
    torch.manual_seed(0)
    m = VisionTransformer(image_size=64, patch_size=8, num_classes=16, embed_dim=256, depth=2, num_heads=4,
                          fp8=True).cuda()
    opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=0.01)
    g = torch.Generator(device="cuda").manual_seed(123)
    X = (torch.rand(256, 3, 64, 64, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    Y = torch.randint(0, 16, (256,), device="cuda", generator=g)
    losses = []
    for i in range(steps):
        idx = torch.arange(64, device="cuda") + 64 * (i % 4)
        opt.zero_grad(set_to_none=True)
        loss = fused.softmax_cross_entropy(m(X[idx]), Y[idx])
        loss.backward()
        opt.step()
        losses.append(loss.detach())
    return torch.stack(losses).float().cpu()


@pytest.mark.timeout(300)
def test_fp8_attention_training_tracks_bf16_attention():
    assert no.available()
    fused.set_backend("native")
    old = os.environ.get("PDT_FP8_ATTN")
    try:
        l8 = _train(True)
        l16 = _train(False)
    finally:
        if old is None:
            os.environ.pop("PDT_FP8_ATTN", None)
        else:
            os.environ["PDT_FP8_ATTN"] = old
        fused.set_backend("auto")
    assert torch.isfinite(l8).all() and torch.isfinite(l16).all()
    w8, w16 = l8[-20:].mean().item(), l16[-20:].mean().item()
    first = l16[:4].mean().item()
    print(f"loss start {first:.3f}; last-20 mean fp8 attention {w8:.4f} vs bf16 attention {w16:.4f}")
    assert w16 < 0.5 * first and w8 < 0.5 * first          # both arms learn the task
    assert abs(w8 - w16) < 0.15 * max(w16, 0.05) + 0.02    # and fp8 attention tracks bf16 attention

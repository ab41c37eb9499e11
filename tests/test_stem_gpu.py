"""Halo-patch ResNet stem kernel (csrc/stem.hip): the 7x7/2 conv over the 4-channel padded
NHWC input and its BatchNorm partial statistics, against an fp32 conv of the same bf16
operands; the persistent band loop runs several bands per workgroup at N = 40 (560 bands)."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_template_amd.ops import native_ops as no

pytestmark = pytest.mark.gpu


def nrmerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("N", [2, 40])
def test_stem_halo_forward_and_stats(N):
    lib = no._load()
    dev = "cuda"
    torch.manual_seed(11)
    H = W = 224
    assert lib.pdt_stem_fwd_rows(N, H, W, 64) > 0
    x = torch.randn(N, 3, H, W, device=dev).to(torch.bfloat16)
    x4 = F.pad(x.permute(0, 2, 3, 1), (0, 1)).contiguous()  # [N][H][W][4] NHWC, channel 3 = 0
    w = torch.randn(64, 3, 7, 7, device=dev) * 0.1
    wb = no._s2d_weight(w)
    y = torch.full((N, H // 2, W // 2, 64), float("nan"), device=dev).to(torch.bfloat16)
    R = lib.pdt_stem_fwd_rows(N, H, W, 64)
    part = torch.full((2 * R * 64,), float("nan"), device=dev)
    rc = lib.pdt_stem_fwd(no._p(x4), no._p(wb), no._p(y), no._p(part), N, H, W, 64, no._s())
    assert rc == 0, rc
    torch.cuda.synchronize()
    ref = F.conv2d(x.float(), w.to(torch.bfloat16).float(), None, 2, 3).permute(0, 2, 3, 1)
    assert nrmerr(y, ref) < 1e-2
    assert torch.isfinite(y.float()).all()
    ps = part.view(2, R, 64).sum(1)
    r2 = ref.reshape(-1, 64)
    assert nrmerr(ps[0], r2.sum(0)) < 1e-3
    assert nrmerr(ps[1], (r2 * r2).sum(0)) < 1e-3


def test_stem_halo_in_the_model_matches_generic(monkeypatch):
    """The stem unit through native_ops (BN statistics -> finalize) gives the same normalised
    statistics whichever kernel computes it."""
    dev = "cuda"
    torch.manual_seed(12)
    N, H = 4, 224
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev).to(memory_format=torch.channels_last)
    bn = torch.nn.BatchNorm2d(64).to(dev)
    x = torch.randn(N, 3, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for halo in ("1", "0"):
        monkeypatch.setenv("PDT_STEM_HALO", halo)
        monkeypatch.setenv("PDT_AUTOTUNE", "0")
        bna = no._BNArgs(bn)
        bna.rm, bna.rv = bn.running_mean.clone(), bn.running_var.clone()
        u = no._unit_fwd_s2d(x, conv.weight, bn.weight, bn.bias, bna)
        outs.append((u.y.float().clone(), u.mean.clone(), u.invstd.clone()))
    assert nrmerr(outs[0][0], outs[1][0]) < 1e-2
    assert nrmerr(outs[0][1], outs[1][1]) < 1e-3
    assert nrmerr(outs[0][2], outs[1][2]) < 1e-3

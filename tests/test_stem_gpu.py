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


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("N", [2, 40])
def test_stem_halo_weight_gradient_with_bn_backward_apply(N, variant):
    """pdt_stem_wgrad (+ pdt_wgrad_reduce) = the stem weight gradient of dy = k1 * relu_gate(dA)
    + k2 * y + k3 (gate from y * scale + shift > 0), dy rounded to bf16 as the kernel stages it."""
    lib = no._load()
    dev = "cuda"
    torch.manual_seed(13)
    H = W = 224
    splits = lib.pdt_stem_wgrad_splits_v(N, H, W, 64, variant)
    assert splits > 0
    x = torch.randn(N, 3, H, W, device=dev).to(torch.bfloat16)
    x4 = F.pad(x.permute(0, 2, 3, 1), (0, 1)).contiguous()
    dA = torch.randn(N, H // 2, W // 2, 64, device=dev).to(torch.bfloat16)
    y = torch.randn(N, H // 2, W // 2, 64, device=dev).to(torch.bfloat16)
    coef = torch.stack([torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1,
                        torch.randn(64, device=dev) * 0.1, torch.rand(64, device=dev) + 0.5,
                        torch.randn(64, device=dev) * 0.2]).contiguous()
    ws = torch.full((lib.pdt_wgrad_workspace(splits, 64, 256),), float("nan"), device=dev)
    dw256 = torch.full((64, 256), float("nan"), device=dev)
    assert lib.pdt_stem_wgrad_v(no._p(x4), no._p(dA), no._p(y), no._p(coef), no._p(ws), N, H, W, 64, variant,
                                no._s()) == 0
    assert lib.pdt_wgrad_reduce(no._p(ws), no._p(dw256), None, None, splits, 64, 256, 1.0, 0, no._s()) == 0
    torch.cuda.synchronize()
    k1, k2, k3, sc, sh = coef
    yf, df = y.float(), dA.float()
    dy = k1 * torch.where(yf * sc + sh > 0, df, torch.zeros_like(df)) + k2 * yf + k3
    dy = dy.to(torch.bfloat16).float().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(x.float(), (64, 3, 7, 7), dy, 2, 3)
    got = no._s2d_unfold_grad(dw256, 3)
    assert torch.isfinite(dw256).all()
    assert nrmerr(got, ref) < 1e-2


def test_stem_pool_backward_fused_bn_reduction():
    """pdt_maxpool_bwd_bnred = pdt_maxpool_bwd (dA, bit for bit) + the stem BN backward partials
    (sum of the ReLU-gated dA and of gated dA * (y - mean)) in one pass."""
    lib = no._load()
    dev = "cuda"
    torch.manual_seed(14)
    N, H, W, C = 6, 112, 112, 64
    Ho, Wo = 56, 56
    y = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    mean = torch.randn(C, device=dev) * 0.1
    scale = torch.rand(C, device=dev) + 0.5
    shift = torch.randn(C, device=dev) * 0.2
    pooled = torch.empty(N, Ho, Wo, C, device=dev, dtype=torch.bfloat16)
    idx = torch.empty(N * Ho * Wo * C, dtype=torch.uint8, device=dev)
    assert lib.pdt_maxpool_fwd_affine(no._p(y), no._p(pooled), no._p(idx), no._p(scale), no._p(shift), N, H, W, C,
                                      Ho, Wo, 3, 2, 1, no._s()) == 0
    dout = torch.randn(N, Ho, Wo, C, device=dev).to(torch.bfloat16)
    dA_ref = torch.empty(N, H, W, C, device=dev, dtype=torch.bfloat16)
    assert lib.pdt_maxpool_bwd(no._p(dout), no._p(idx), no._p(dA_ref), N, H, W, C, Ho, Wo, 3, 2, 1, no._s()) == 0
    blocks = 200
    part = torch.full((2 * blocks * C,), float("nan"), device=dev)
    dA = torch.empty_like(dA_ref)
    assert lib.pdt_maxpool_bwd_bnred(no._p(dout), no._p(idx), no._p(dA), no._p(y), no._p(mean), no._p(scale),
                                     no._p(shift), no._p(part), N, H, W, C, Ho, Wo, blocks, no._s()) == 0
    torch.cuda.synchronize()
    assert torch.equal(dA, dA_ref)
    yf = y.float()
    g = torch.where(yf * scale + shift > 0, dA_ref.float(), torch.zeros_like(yf)).reshape(-1, C)
    ps = part.view(2, blocks, C).sum(1)
    assert nrmerr(ps[0], g.sum(0)) < 1e-4
    assert nrmerr(ps[1], (g * (yf.reshape(-1, C) - mean)).sum(0)) < 1e-4

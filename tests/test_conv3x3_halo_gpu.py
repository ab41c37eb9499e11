"""The stride-1 3x3 halo-patch implicit GEMM (csrc/conv3x3_halo.hip) against fp32
PyTorch references: forward output + BatchNorm statistics partials, data gradient,
and the data gradient's fused BatchNorm-backward partials -- for every halo variant,
on tiles that straddle images and a partial last tile."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def relerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _halo_variants():
    lib = no._load()
    return [v for v in range(lib.pdt_conv_nt_num_variants()) if lib.pdt_conv_nt_variant_kind(v) == 2]


SHAPES = [  # N, Cin, H, W, Cout
    (2, 64, 56, 56, 64),     # stage 1: one 64-channel chunk, 4 rows per tile
    (3, 128, 28, 28, 128),   # 8 rows per tile: tiles straddle images, partial last tile
    (5, 256, 14, 14, 256),   # 16 rows per tile, 4 chunks
    (2, 64, 14, 14, 128),
]


@pytest.mark.parametrize("shape", SHAPES)
def test_halo_forward_and_stats(shape):
    torch.manual_seed(0)
    N, Cin, H, W, Cout = shape
    lib = no._load()
    x = _cl(torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16))
    w = _cl(torch.randn(Cout, Cin, 3, 3, device="cuda") * (2.0 / (9 * Cin)) ** 0.5)
    wb = no.bf16_weight(w)
    ref = F.conv2d(x.float(), w.to(torch.bfloat16).float(), None, 1, 1)
    g = dict(KH=3, KW=3, sh=1, sw=1, ph=1, pw=1, Ho=H, Wo=W)
    a = no._fwd_nt_geom(N, H, W, Cin, Cout, g)
    M = N * H * W
    ran = 0
    for v in _halo_variants():
        rows = lib.pdt_conv_nt_stat_rows(M, Cout, a["K"], v)
        part = torch.full((2 * rows * Cout,), float("nan"), device="cuda")
        y = torch.full_like(ref, float("nan"), dtype=torch.bfloat16, memory_format=torch.channels_last)
        rc = lib.pdt_conv_nt(*no._nt_args(x, wb, y, part, None, a, 0, v))
        if rc == no.NOT_APPLICABLE:
            continue
        assert rc == 0, (v, rc)
        ran += 1
        assert relerr(y, ref) < 1e-2, v
        ps = part.view(2, rows, Cout).sum(1)
        assert relerr(ps[0], ref.sum((0, 2, 3))) < 2e-3, v
        assert relerr(ps[1], (ref * ref).sum((0, 2, 3))) < 2e-3, v
    assert ran >= 1


@pytest.mark.parametrize("gate_mode", ["y", "mask", "none"])
@pytest.mark.parametrize("shape", SHAPES)
def test_halo_dgrad_and_fused_bn_backward_partials(shape, gate_mode):
    """The halo data gradient with the fused BN-backward partials, for each compiled ReLU gate
    (recomputed from y, the unit's bit mask, no ReLU) vs fp32."""
    torch.manual_seed(1)
    N, Cin, H, W, Cout = shape
    lib = no._load()
    w = _cl(torch.randn(Cout, Cin, 3, 3, device="cuda") * (2.0 / (9 * Cin)) ** 0.5)
    dy = _cl(torch.randn(N, Cout, H, W, device="cuda").to(torch.bfloat16))
    wr = w.to(torch.bfloat16).float()
    rdx = torch.nn.grad.conv2d_input((N, Cin, H, W), wr, dy.float(), 1, 1)
    # the dgrad geometry _conv_dgrad builds for a stride-1 3x3 conv (one phase)
    wt = torch.empty(Cin * 9 * Cout, dtype=torch.bfloat16, device="cuda")
    no._chk(lib.pdt_wt_dgrad(no._p(w), no._p(wt), Cout, 3, 3, Cin, 0, 0, 1, 3, 3, no._s()), "wt")
    a = dict(Hs=H, Ws=W, Cs=Cout, Nimg=N, Hm=H, Wm=W, Ncol=Cin, K=9 * Cout, ldb=9 * Cout, sh=1, sw=1, oh0=1,
             ow0=1, dh=-1, dw=-1, nth=3, ntw=3, Ho=H, Wo=W, osh=1, osw=1, oph=0, opw=0, ldo=Cin)
    # the BN(+ReLU) unit the data gradient feeds: y (its pre-BN output), mean, scale, shift
    yb = _cl(torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16))
    mean = torch.randn(Cin, device="cuda") * 0.1
    scale = torch.rand(Cin, device="cuda") + 0.5
    shift = torch.randn(Cin, device="cuda") * 0.1
    M = N * H * W
    bmask = torch.randint(0, 256, (M * Cin // 8,), dtype=torch.uint8, device="cuda") if gate_mode == "mask" else None
    ran = 0
    for v in _halo_variants():
        dx = torch.full_like(yb, float("nan"))
        rc = lib.pdt_conv_nt(*no._nt_args(dy, wt, dx, None, None, a, 0, v))
        if rc == no.NOT_APPLICABLE:
            continue
        assert rc == 0, (v, rc)
        ran += 1
        assert relerr(dx, rdx) < 1e-2, v
        R = lib.pdt_conv_nt_bnb_rows(M, Cin, a["K"], v)
        part = torch.full((2 * R * Cin,), float("nan"), device="cuda")
        dx2 = torch.full_like(yb, float("nan"))
        rc = lib.pdt_conv_nt_bnb(
            no._p(dy), no._p(wt), no._p(dx2), None, None, a["Hs"], a["Ws"], a["Cs"], a["Nimg"], a["Hm"], a["Wm"],
            a["Ncol"], a["K"], a["ldb"], a["sh"], a["sw"], a["oh0"], a["ow0"], a["dh"], a["dw"], a["nth"], a["ntw"],
            a["Ho"], a["Wo"], a["osh"], a["osw"], a["oph"], a["opw"], a["ldo"], v, no._p(yb), no._p(mean),
            no._p(scale), no._p(shift), no._p(bmask), no._p(part), int(gate_mode != "none"), 0, R, no._s())
        assert rc == 0, (v, rc)
        assert torch.equal(dx2, dx), v  # same stored gradient
        yf = yb.float()
        if gate_mode == "y":
            gate = (yf * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)) > 0
        elif gate_mode == "mask":  # bit k of byte i gates element 8 i + k of the NHWC storage
            bits = ((bmask.view(-1, 1).int() >> torch.arange(8, device="cuda")) & 1).view(N, H, W, Cin)
            gate = bits.permute(0, 3, 1, 2).bool()
        else:
            gate = torch.ones_like(yf, dtype=torch.bool)
        gq = dx.float() * gate
        ps = part.view(2, R, Cin).sum(1)
        assert relerr(ps[0], gq.sum((0, 2, 3))) < 2e-3, v
        assert relerr(ps[1], (gq * (yf - mean.view(1, -1, 1, 1))).sum((0, 2, 3))) < 2e-3, v
    assert ran >= 1


@pytest.mark.parametrize("shape", SHAPES)
def test_halo_wgrad(shape):
    torch.manual_seed(2)
    N, Cin, H, W, Cout = shape
    lib = no._load()
    x = _cl(torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16))
    dy = _cl(torch.randn(N, Cout, H, W, device="cuda").to(torch.bfloat16))
    ref = torch.nn.grad.conv2d_weight(x.float(), (Cout, Cin, 3, 3), dy.float(), 1, 1)
    wa = dict(M=N * H * W, Mo=Cout, No=9 * Cin, ldy=Cout, Hs=H, Ws=W, C=Cin, Hm=H, Wm=W, sh=1, sw=1, oh0=-1, ow0=-1,
              dh=1, dw=1, ntw=3)
    hv = lib.pdt_wgrad_halo_id()
    dw = torch.full((Cout, Cin, 3, 3), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
    rc = no._wgrad_launch(lib, dy, x, dw, hv, 1.0, False, wa)
    assert rc == 0, rc
    assert relerr(dw, ref) < 1e-2
    # accumulate mode adds onto the existing gradient
    rc = no._wgrad_launch(lib, dy, x, dw, hv, 1.0, True, wa)
    assert rc == 0 and relerr(dw, 2 * ref) < 1e-2

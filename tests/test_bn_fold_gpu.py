"""BatchNorm applies folded into the A staging of the consuming 1x1 GEMM
(csrc/conv_nt_kernel.h AXArgs, csrc/conv_igemm_ax.hip):

* the tensor the fold writes for its other consumers (the block output + ReLU bit mask
  in the forward; dy3 in the backward) equals the element pass (csrc/bn_act.hip) it
  replaces to within one bf16 rounding (the two kernels may contract the same fp32
  expression into FMAs differently), for every AX tile;
* the GEMM output equals the unfused GEMM on the element pass's output;
* a whole identity bottleneck's backward with the fold on matches the fold off;
* a bottleneck chain (the ResNet path: every block's output BN pass deferred into the
  next block's conv1, incl. the downsample blocks' affine residual), training and eval,
  matches the unfolded blocks.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def assert_one_rounding(a, b, what):
    """a, b: bf16 results of the same fp32 expression: equal up to one bf16 ulp of the result."""
    a, b = a.float(), b.float()
    bad = ((a - b).abs() > b.abs() * 2.0 ** -7 + 1e-5).sum().item()
    assert bad == 0, (what, bad)


def nrmerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


@pytest.mark.parametrize("C,Cm,H", [(256, 64, 14), (512, 128, 7)])
def test_ax_mode2_dy3_and_dgrad(C, Cm, H):
    """mode 2: dy3 = k1*gate(dout) + k2*y3 + k3 staged and written by conv3's dgrad."""
    torch.manual_seed(0)
    lib = no._load()
    N = 6
    dout = _cl(torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16))
    y3 = _cl(torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16))
    mask = torch.randint(0, 256, (dout.numel() // 8,), dtype=torch.uint8, device="cuda")
    k1, k2, k3 = (torch.randn(C, device="cuda") for _ in range(3))
    # reference: the element pass, then the plain data gradient
    dy_ref = torch.empty_like(y3)
    no._chk(lib.pdt_bn_bwd_apply(no._p(dout), no._p(y3), None, None, None, no._p(k1), no._p(k2), no._p(k3),
                                 no._p(dy_ref), None, y3.numel() // C, C, 1, no._p(mask), no._s()), "apply")
    w = _cl(torch.randn(C, Cm, 1, 1, device="cuda") * 0.05)
    wt = torch.empty(Cm * C, dtype=torch.bfloat16, device="cuda")
    no._chk(lib.pdt_wt_dgrad(no._p(w), no._p(wt), C, 1, 1, Cm, 0, 0, 1, 1, 1, no._s()), "wt")
    ref = torch.nn.functional.conv2d(dy_ref.float(), w.detach().to(torch.bfloat16).float().transpose(0, 1))
    a = dict(Hs=H, Ws=H, Cs=C, Nimg=N, Hm=H, Wm=H, Ncol=Cm, K=C, ldb=C, ldo=Cm)
    yb = _cl(torch.randn(N, Cm, H, H, device="cuda").to(torch.bfloat16))
    mean, sc, sh = torch.zeros(Cm, device="cuda"), torch.ones(Cm, device="cuda"), torch.zeros(Cm, device="cuda")
    M = N * H * H
    ran = 0
    for v in no.AX_VARIANTS:
        R = lib.pdt_conv_nt_bnb_rows(M, Cm, C, v)
        part = torch.empty(2 * R * Cm, device="cuda")
        dy = torch.full_like(y3, float("nan"))
        out = torch.full_like(yb, float("nan"))
        rc = no._ax_launch(lib, dout, wt, out, v, a, bnb=(yb, mean, sc, sh, None, part, 1, 0, R),
                           ax=(2, y3, k1, k2, k3, None, None, mask, None, dy))
        assert rc == 0, (v, rc)
        ran += 1
        assert_one_rounding(dy, dy_ref, v)
        assert nrmerr(out, ref) < 1e-2, v
    assert ran == len(no.AX_VARIANTS)


@pytest.mark.parametrize("affine_res", [False, True])
def test_ax_mode1_out_mask_and_fwd(affine_res):
    """mode 1: out = relu(y3*s + b + res) (+ the downsample BN affine on res) staged and
    written by the next conv1, with its ReLU bit mask."""
    torch.manual_seed(1)
    lib = no._load()
    N, C, Cm, H = 6, 256, 64, 14
    y3 = _cl(torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16))
    res = _cl(torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16))
    s, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    rs, rb = (torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1) if affine_res else (None, None)
    out_ref = torch.empty_like(y3)
    mask_ref = torch.empty(y3.numel() // 8, dtype=torch.uint8, device="cuda")
    M = N * H * H
    if affine_res:
        no._chk(lib.pdt_bn_apply_res_affine(no._p(y3), no._p(res), no._p(out_ref), no._p(s), no._p(b), no._p(rs),
                                            no._p(rb), M, C, 1, no._p(mask_ref), no._s()), "apply")
    else:
        no._chk(lib.pdt_bn_apply(no._p(y3), no._p(res), no._p(out_ref), no._p(s), no._p(b), M, C, 1,
                                 no._p(mask_ref), no._s()), "apply")
    w = _cl(torch.randn(Cm, C, 1, 1, device="cuda") * 0.05)
    wb = no.bf16_weight(w)
    ref = torch.nn.functional.conv2d(out_ref.float(), w.to(torch.bfloat16).float())
    a = dict(Hs=H, Ws=H, Cs=C, Nimg=N, Hm=H, Wm=H, Ncol=Cm, K=C, ldb=C, ldo=Cm)
    for v in no.AX_VARIANTS:
        rows = lib.pdt_conv_nt_stat_rows(M, Cm, C, v)
        st = torch.empty(2 * rows * Cm, device="cuda")
        out = torch.full_like(y3, float("nan"))
        mk = torch.zeros_like(mask_ref)
        y1 = _cl(torch.empty(N, Cm, H, H, device="cuda", dtype=torch.bfloat16))
        rc = no._ax_launch(lib, y3, wb, y1, v, a, stats=st, ax=(1, res, s, b, None, rs, rb, None, mk, out))
        assert rc == 0, (v, rc)
        assert_one_rounding(out, out_ref, v)
        flips = (mk ^ mask_ref).to(torch.int32)
        assert int(sum(((flips >> k) & 1).sum().item() for k in range(8))) <= 4, v  # only at a rounding tie with 0
        assert nrmerr(y1, ref) < 1e-2, v
        ps = st.view(2, rows, Cm).sum(1)
        assert nrmerr(ps[0], ref.sum((0, 2, 3))) < 2e-3, v


def test_identity_bottleneck_backward_with_and_without_fold(monkeypatch):
    from pytorch_distributed_template_amd.models.resnet import Bottleneck
    torch.manual_seed(7)
    blk = Bottleneck(256, 64).cuda().to(memory_format=torch.channels_last)
    x = _cl(torch.randn(8, 256, 14, 14, device="cuda").to(torch.bfloat16))
    g = _cl(torch.randn(8, 256, 14, 14, device="cuda").to(torch.bfloat16))
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("PDT_FUSE_BN_AX", on)
        for p in blk.parameters():
            p.grad = None
        xi = x.detach().clone().requires_grad_(True)
        y = no.bottleneck(xi, blk)
        y.backward(g)
        res.append((y.detach().float(), xi.grad.float(), [p.grad.float().clone() for p in blk.parameters()]))
    (y1, dx1, g1), (y0, dx0, g0) = res
    assert nrmerr(y1, y0) < 1e-3  # bn2's apply folded into conv3: one bf16 rounding apart at most
    assert nrmerr(dx1, dx0) < 2e-3
    for a, b in zip(g1, g0):
        assert nrmerr(a, b) < 2e-3


def _chain():
    from pytorch_distributed_template_amd.models.resnet import Bottleneck
    return torch.nn.Sequential(Bottleneck(64, 64, 1, downsample=True), Bottleneck(256, 64),
                               Bottleneck(256, 128, 2, downsample=True), Bottleneck(512, 128)).cuda().to(
        memory_format=torch.channels_last)


@pytest.mark.parametrize("force", [None, 5, 25])
@pytest.mark.parametrize("train", [True, False])
def test_bottleneck_chain_fold_matches_unfolded(monkeypatch, train, force):
    """Fold on vs off, both against the fp32 stock-op reference of the same chain: the fold
    may flip bf16 roundings (which small-batch BatchNorms re-normalise and the backward
    amplifies), so the check is that it is no less accurate than the unfolded blocks.
    ``force``: every fold site takes AX tile ``force`` (5: register-staged 128x128, 25: the
    LDS-DMA 128x128) instead of the tuner's choice, so the 1x1 and 3x3 folds (forward modes
    with and without residual, backward modes 2 and 3) all run whatever the timings say."""
    if force is not None:
        monkeypatch.setattr(no, "_ax_select", lambda key, run, run_ref=None: force)
    from pytorch_distributed_template_amd.ops import fused
    torch.manual_seed(11)
    net = _chain()
    net.train(train)
    state = {k: v.clone() for k, v in net.state_dict().items()}
    x = _cl(torch.randn(8, 64, 16, 16, device="cuda").to(torch.bfloat16))
    gy = None
    res = []
    try:
        for arm in ("1", "0", "ref"):
            net.load_state_dict(state)
            for p in net.parameters():
                p.grad = None
            if arm == "ref":
                fused.set_backend("torch")
                xi = x.detach().float().requires_grad_(train)
                y = fused.bottleneck_chain(xi, list(net))
            else:
                fused.set_backend("native")
                monkeypatch.setenv("PDT_FUSE_BN_AX", arm)
                xi = x.detach().clone().requires_grad_(train)
                y = fused.bottleneck_chain(xi, list(net))
            grads = []
            if train:
                if gy is None:
                    gy = _cl(torch.randn(y.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(3))
                             .to(torch.bfloat16))
                y.backward(gy.to(y.dtype))
                grads = [xi.grad.float()] + [p.grad.float().clone() for p in net.parameters()]
            bufs = [b.float().clone() for n, b in net.named_buffers() if "running" in n]
            res.append((y.detach().float(), grads, bufs))
    finally:
        fused.set_backend("auto")
    (y1, g1, b1), (y0, g0, b0), (yr, gr, br) = res
    assert torch.isfinite(y1).all()
    e1, e0 = nrmerr(y1, yr), nrmerr(y0, yr)
    assert e1 <= 1.5 * e0 + 2e-3, (e1, e0)
    for i, (a, b, r) in enumerate(zip(g1, g0, gr)):
        e1, e0 = nrmerr(a, r), nrmerr(b, r)
        assert e1 <= 1.5 * e0 + 5e-3, (i, e1, e0)
    for a, b, r in zip(b1, b0, br):
        assert nrmerr(a, r) <= 1.5 * nrmerr(b, r) + 1e-3


def test_ax_mode3_conv1_dgrad_with_addend():
    """mode 3 on a 1x1 geometry with an addend: a bottleneck's conv1 data gradient with bn1's
    backward apply in its A staging (ReLU gate recomputed from y1), the shortcut gradient
    (masked by the block's ReLU bits) added in the epilogue, and the previous block's bn3
    backward partials (gated by its ReLU bit mask) -- against the element pass followed by
    the plain fused-epilogue data gradient (``pdt_conv_nt_bnb``), for every AX tile."""
    torch.manual_seed(5)
    lib = no._load()
    N, Cin, C1, H = 6, 256, 64, 14
    M = N * H * H
    da1 = _cl(torch.randn(N, C1, H, H, device="cuda").to(torch.bfloat16))
    y1 = _cl(torch.randn(N, C1, H, H, device="cuda").to(torch.bfloat16))
    sc1, sh1 = torch.rand(C1, device="cuda") + 0.5, torch.randn(C1, device="cuda") * 0.2
    k1, k2, k3 = (torch.randn(C1, device="cuda") for _ in range(3))
    dy_ref = torch.empty_like(y1)
    no._chk(lib.pdt_bn_bwd_apply(no._p(da1), no._p(y1), None, no._p(sc1), no._p(sh1), no._p(k1), no._p(k2),
                                 no._p(k3), no._p(dy_ref), None, M, C1, 1, None, no._s()), "apply")
    w = _cl(torch.randn(C1, Cin, 1, 1, device="cuda") * 0.05)
    wt = torch.empty(Cin * C1, dtype=torch.bfloat16, device="cuda")
    no._chk(lib.pdt_wt_dgrad(no._p(w), no._p(wt), C1, 1, 1, Cin, 0, 0, 1, 1, 1, no._s()), "wt")
    addend = _cl(torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16))
    amask = torch.randint(0, 256, (addend.numel() // 8,), dtype=torch.uint8, device="cuda")
    yp = _cl(torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16))
    pmask = torch.randint(0, 256, (yp.numel() // 8,), dtype=torch.uint8, device="cuda")
    mean = torch.randn(Cin, device="cuda") * 0.1
    a = dict(Hs=H, Ws=H, Cs=C1, Nimg=N, Hm=H, Wm=H, Ncol=Cin, K=C1, ldb=C1, sh=1, sw=1, oh0=0, ow0=0, dh=-1, dw=-1,
             nth=1, ntw=1, Ho=H, Wo=H, osh=1, osw=1, oph=0, opw=0, ldo=Cin)
    Rr = lib.pdt_conv_nt_bnb_rows(M, Cin, C1, 0)
    part_ref = torch.empty(2 * Rr * Cin, device="cuda")
    out_ref = torch.empty_like(addend)
    no._chk(lib.pdt_conv_nt_bnb(no._p(dy_ref), no._p(wt), no._p(out_ref), no._p(addend), no._p(amask), H, H, C1, N,
                                H, H, Cin, C1, C1, 1, 1, 0, 0, -1, -1, 1, 1, H, H, 1, 1, 0, 0, Cin, 0, no._p(yp),
                                no._p(mean), None, None, no._p(pmask), no._p(part_ref), 1, 0, Rr, no._s()), "bnb ref")
    sums_ref = part_ref.view(2, Rr, Cin).sum(1)
    ran = 0
    for v in no.AX_VARIANTS:
        R = lib.pdt_conv_nt_bnb_rows(M, Cin, C1, v)
        part = torch.empty(2 * R * Cin, device="cuda")
        dy = torch.full_like(y1, float("nan"))
        out = torch.full_like(addend, float("nan"))
        rc = no._ax2_launch(lib, da1, wt, out, v, a, bnb=(yp, mean, None, None, pmask, part, 1, 0, R),
                            ax=(3, y1, k1, k2, k3, sc1, sh1, None, None, dy), addend=addend, addend_mask=amask)
        if rc == no.NOT_APPLICABLE:
            continue
        assert rc == 0, (v, rc)
        ran += 1
        assert_one_rounding(dy, dy_ref, v)
        assert nrmerr(out, out_ref) < 1e-2, v
        assert nrmerr(part.view(2, R, Cin).sum(1), sums_ref) < 1e-2, v
    assert ran >= len(no.AX_VARIANTS) - 3


class _FakeUnit:
    def __init__(self, y, mean, scale=None, shift=None, relu=True):
        self.y, self.mean, self.scale, self.shift, self.relu = y, mean, scale, shift, relu
        self.Cout = y.shape[1]


@pytest.mark.parametrize("v,with_add", [(5, False), (15, False), (25, False), (27, False), (38, False), (40, False),
                                        (37, False), (37, True), (36, True)])
def test_dgrad_epilogue_second_unit_partials(monkeypatch, v, with_add):
    """A data-gradient epilogue producing the BN-backward partials of TWO units fed by the
    same ReLU-gated gradient (a downsample block's bn3 and shortcut BN): both partial sets
    against fp32 sums over the stored gradient. A ring tile (36, 37) compiles no second unit:
    given a block input (addend + mask) it runs the single-unit epilogue (second = None);
    given a configuration it does not compile at all (mask without addend) the launch moves
    to the generic tile, which carries both units."""
    torch.manual_seed(v)
    N, Cin, Cm, H = 4, 256, 64, 14
    dy = _cl(torch.randn(N, Cm, H, H, device="cuda").to(torch.bfloat16))
    w = _cl(torch.randn(Cm, Cin, 1, 1, device="cuda") * 0.05)
    y3 = _cl(torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16))
    yd = _cl(torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16))
    m3, md = torch.randn(Cin, device="cuda") * 0.1, torch.randn(Cin, device="cuda") * 0.1
    mask = torch.randint(0, 256, (y3.numel() // 8,), dtype=torch.uint8, device="cuda")
    u3, ud = _FakeUnit(y3, m3), _FakeUnit(yd, md, relu=False)
    monkeypatch.setattr(no, "_select_bnb_variant", lambda *a, **k: v)
    g = {"KH": 1, "KW": 1, "sh": 1, "sw": 1, "ph": 0, "pw": 0, "Ho": H, "Wo": H}
    add = _cl(torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16)) if with_add else None
    dx, pre = no._conv_dgrad(dy, w, N, H, H, Cin, Cm, g, addend=add, bnb_unit=u3, bnb_mask=mask, bnb_unit2=ud)
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv2d(dy.float(), w.to(torch.bfloat16).float().transpose(0, 1))
    if with_add:
        ref = ref + add.float()
    assert nrmerr(dx, ref) < 1e-2
    bits = torch.stack([(mask >> k) & 1 for k in range(8)], 1).reshape(-1).bool()
    gate = dx.float().permute(0, 2, 3, 1).reshape(-1, Cin) * bits.view(-1, Cin)
    s_ref = gate.sum(0)
    q3_ref = (gate * (y3.float().permute(0, 2, 3, 1).reshape(-1, Cin) - m3)).sum(0)
    qd_ref = (gate * (yd.float().permute(0, 2, 3, 1).reshape(-1, Cin) - md)).sum(0)
    R = pre.R
    p3 = pre.part[:2 * R * Cin].view(2, R, Cin).sum(1)
    assert nrmerr(p3[0], s_ref) < 1e-3 and nrmerr(p3[1], q3_ref) < 1e-3
    if v in (36, 37) and with_add:
        assert pre.second is None
        return
    assert pre.second is not None and pre.second.unit is ud
    pd = pre.second.part[:2 * R * Cin].view(2, R, Cin).sum(1)
    assert nrmerr(pd[0], s_ref) < 1e-3 and nrmerr(pd[1], qd_ref) < 1e-3


@pytest.mark.parametrize("geom", ["3x3", "stem_s2d"])
def test_wgrad_bn_backward_apply_in_staging(geom):
    """The weight gradient forming dY = k1*gate(dA) + k2*y + k3 while staging dA
    (pdt_conv_wgrad2; the stem's BN backward apply) against the element pass followed by
    the plain weight gradient, for every tile that carries it."""
    torch.manual_seed(3)
    lib = no._load()
    if geom == "3x3":
        N, C, Co, H = 4, 64, 64, 14
        x = _cl(torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16))
        a = dict(M=N * H * H, Mo=Co, No=9 * C, ldy=Co, Hs=H, Ws=H, C=C, Hm=H, Wm=H, sh=1, sw=1, oh0=-1, ow0=-1,
                 dh=1, dw=1, ntw=3)
        shp = (N, Co, H, H)
    else:  # the space-to-depth stem: NHWC padded to 4 channels, 8 x 4 taps of 8 "channels"
        N, Co, H = 2, 64, 224
        x = torch.zeros(N, H, H, 4, device="cuda", dtype=torch.bfloat16)
        x[..., :3] = torch.randn(N, H, H, 3, device="cuda").to(torch.bfloat16)
        a = dict(M=N * 112 * 112, Mo=Co, No=256, ldy=Co, Hs=H, Ws=H, C=8, Hm=112, Wm=112, sh=2, sw=2, oh0=-3,
                 ow0=-4, dh=1, dw=2, ntw=4, pix=4)
        shp = (N, Co, 112, 112)
    dA = _cl(torch.randn(shp, device="cuda").to(torch.bfloat16))
    y = _cl(torch.randn(shp, device="cuda").to(torch.bfloat16))
    k1, k2, k3 = (torch.randn(Co, device="cuda") * 0.5 for _ in range(3))
    sc, sh = torch.rand(Co, device="cuda") + 0.5, torch.randn(Co, device="cuda") * 0.2
    coef = torch.stack([k1, k2, k3, sc, sh]).contiguous()
    dy = torch.empty_like(y)
    no._chk(lib.pdt_bn_bwd_apply(no._p(dA), no._p(y), None, no._p(sc), no._p(sh), no._p(k1), no._p(k2), no._p(k3),
                                 no._p(dy), None, y.numel() // Co, Co, 1, None, no._s()), "apply")
    ran = 0
    for v in no.WGB_VARIANTS:
        ref = torch.zeros(Co * a["No"], device="cuda")
        got = torch.full_like(ref, float("nan"))
        assert no._wgrad_launch(lib, dy, x, ref, v, 1.0, False, a) == 0
        rc = no._wgrad_launch(lib, dA, x, got, v, 1.0, False, a, bna=(y, coef))
        assert rc == 0, (v, rc)
        ran += 1
        assert nrmerr(got, ref) < 2e-3, (v, nrmerr(got, ref))
    assert ran == len(no.WGB_VARIANTS)

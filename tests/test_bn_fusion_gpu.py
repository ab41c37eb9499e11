"""BatchNorm-backward reduction fused into the data-gradient GEMM epilogue
(``BnbArgs`` in csrc/conv_igemm.hip, ``_Bottleneck.backward`` in
ops/native_ops.py): fused vs the separate reduce pass vs an fp32 PyTorch
reference of the same ResNet stage. Run on an MI355X."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def nrmerr(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def setup_module(module):
    assert no.available(), "native library must be built and loaded on GPU runs"
    no.require()


def _ref_bottleneck(x, blk):
    """fp32 PyTorch reference of a training-mode bottleneck (batch statistics)."""
    def cb(t, conv, bn, relu):
        t = F.conv2d(t, conv.weight, None, conv.stride, conv.padding)
        t = F.batch_norm(t, None, None, bn.weight, bn.bias, True, 0.0, bn.eps)
        return F.relu(t) if relu else t
    idn = cb(x, blk.downsample[0], blk.downsample[1], False) if blk.downsample is not None else x
    o = cb(x, blk.conv1, blk.bn1, True)
    o = cb(o, blk.conv2, blk.bn2, True)
    return F.relu(cb(o, blk.conv3, blk.bn3, False) + idn)


def _stage():
    from pytorch_distributed_template_amd.models.resnet import Bottleneck
    return nn.Sequential(Bottleneck(256, 128, stride=2, downsample=True), Bottleneck(512, 128),
                         Bottleneck(512, 128))


def test_bn_backward_reduction_fused_into_dgrad_epilogue(monkeypatch):
    """A 3-block stage (stride-2 + downsample, then identity blocks): the BN
    backward reductions computed in the data-gradient epilogues (in-block bn1/bn2,
    and the previous block's bn3 from the next block's input-gradient GEMM) must
    match the separate reduce pass and an fp32 PyTorch reference."""
    torch.manual_seed(11)
    stage = _stage().cuda().to(memory_format=torch.channels_last)
    for m in stage.modules():
        if isinstance(m, nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    x = _cl(torch.randn(8, 256, 28, 28, device="cuda").to(torch.bfloat16))
    gy = _cl(torch.randn(8, 512, 14, 14, device="cuda", generator=torch.Generator("cuda").manual_seed(5))
             .to(torch.bfloat16))
    lib = no._load()
    calls = {"bnb": 0, "reduce": 0}
    orig_bnb, orig_red = lib.pdt_conv_nt_bnb, lib.pdt_bn_bwd_reduce

    def count(name, fn):
        def w(*a):
            calls[name] += 1
            return fn(*a)
        return w
    monkeypatch.setattr(lib, "pdt_conv_nt_bnb", count("bnb", orig_bnb))
    monkeypatch.setattr(lib, "pdt_bn_bwd_reduce", count("reduce", orig_red))

    res = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("PDT_FUSE_BN_BWD", fuse)
        calls.update(bnb=0, reduce=0)
        for p in stage.parameters():
            p.grad = None
        xi = x.detach().clone().requires_grad_(True)
        y = stage(xi)
        y.backward(gy)
        torch.cuda.synchronize()
        res[fuse] = (y.float(), xi.grad.float(), [p.grad.float().clone() for p in stage.parameters()], dict(calls))
    # fused: bn1/bn2 of all 3 blocks + bn3 of blocks 0 and 1 (3x3 s2 dgrad = 4 phase launches);
    # left on the reduce pass: the last block's bn3 and the downsample BN
    assert res["1"][3]["reduce"] == 2, res["1"][3]
    assert res["1"][3]["bnb"] >= 8, res["1"][3]
    assert res["0"][3]["bnb"] == 0 and res["0"][3]["reduce"] == 10, res["0"][3]
    (y1, dx1, g1, _), (y0, dx0, g0, _) = res["1"], res["0"]
    assert nrmerr(y1, y0) == 0.0
    assert nrmerr(dx1, dx0) < 2e-2
    # fp32 reference of the same stage: the fused path must be as accurate as the
    # separate reduce pass (both differ from fp32 only by bf16 rounding, which the
    # BN backward's mean subtraction amplifies through the 3 blocks)
    ref = _stage().cuda()
    with torch.no_grad():
        for q, p in zip(ref.parameters(), stage.parameters()):
            q.copy_(p.float())
    xr = x.detach().float().requires_grad_(True)
    yr = xr
    for blk in ref:
        yr = _ref_bottleneck(yr, blk)
    yr.backward(gy.float())
    e1, e0 = nrmerr(dx1, xr.grad), nrmerr(dx0, xr.grad)
    print(f"dx err vs fp32: fused {e1:.4g} unfused {e0:.4g}; fused vs unfused {nrmerr(dx1, dx0):.4g}")
    assert nrmerr(y1, yr) < 2e-2
    assert e1 < 1.25 * e0 + 2e-3, (e1, e0)
    for a, b, q in zip(g1, g0, ref.parameters()):
        ea, eb = nrmerr(a, q.grad), nrmerr(b, q.grad)
        print(f"  {tuple(a.shape)}: fused {ea:.4g} unfused {eb:.4g}")
        assert ea < 1.25 * eb + 2e-3, (a.shape, ea, eb)


def test_stem_bn_relu_folded_into_maxpool():
    """ResNet stem: max_pool(relu(bn(conv(x)))) with the BN apply done inside the
    max-pool vs the unfused composition (conv_bn_act + max_pool2d) and an fp32
    PyTorch reference. The fused pool compares fp32 values where the unfused one
    compares bf16-rounded activations, so argmax ties resolve differently and the
    gradient of a tied window reaches a different pixel: both are judged against
    the fp32 reference instead of against each other."""
    import torch.nn.functional as F
    torch.manual_seed(3)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda().to(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(64).cuda()
    with torch.no_grad():
        bn.weight.uniform_(-1.0, 1.5)  # negative scales: the affine is not monotonic
        bn.bias.uniform_(-0.3, 0.3)
        conv.weight.copy_(conv.weight.to(torch.bfloat16).float())
    x = _cl(torch.randn(4, 3, 64, 64, device="cuda").to(torch.bfloat16))
    g = None
    res = []
    for path in ("fused", "unfused", "fp32"):
        for p_ in (conv.weight, bn.weight, bn.bias):
            p_.grad = None
        if path == "fused":
            y = no.stem_pool(x, conv, bn)
            assert y is not None
        elif path == "unfused":
            y = no.max_pool2d(no.conv_bn_act(x, conv, bn, relu=True), 3, 2, 1)
        else:
            t = F.conv2d(x.float(), conv.weight, None, 2, 3)
            t = F.relu(F.batch_norm(t, None, None, bn.weight, bn.bias, True, 0.0, bn.eps))
            y = F.max_pool2d(t, 3, 2, 1)
        if g is None:
            g = _cl(torch.randn(y.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(9))
                    .to(torch.bfloat16))
        y.backward(g.to(y.dtype))
        torch.cuda.synchronize()
        res.append((y.float(), conv.weight.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone()))
    fused, unfused, ref = res
    assert fused[0].shape == (4, 64, 16, 16)
    assert nrmerr(fused[0], unfused[0]) < 2e-3
    for k in range(4):
        ef, eu = nrmerr(fused[k], ref[k]), nrmerr(unfused[k], ref[k])
        print(f"stem output/grad {k}: fused {ef:.4g} unfused {eu:.4g}")
        assert ef < 1.25 * eu + 5e-3, (k, ef, eu)


@pytest.mark.parametrize("loader_padded", [False, True])
def test_stem_space_to_depth_vs_direct(monkeypatch, loader_padded):
    """Space-to-depth stem GEMM (K = 8x4 taps of 2 pixels x 4 channels = 256, read
    from NHWC storage padded to 4 channels) vs the direct 7x7 implicit GEMM (49 taps
    of 8 padded channels) and an fp32 PyTorch reference: forward output, conv
    weight gradient and BN gradients. ``loader_padded`` feeds the loader's padded
    NHWC view (read in place) instead of a plain channels_last tensor."""
    torch.manual_seed(5)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda().to(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(64).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
        conv.weight.copy_(conv.weight.to(torch.bfloat16).float())
    if loader_padded:
        from pytorch_distributed_template_amd.data.synthetic import SyntheticImageLoader
        dl = SyntheticImageLoader(batch_size=4, num_samples=4, pool=1, image_size=96, training=False,
                                     device=torch.device("cuda"), dtype=torch.bfloat16)
        x = next(iter(dl))[0]
        assert no.nhwc_padded_view(x, 4) is not None
    else:
        x = _cl(torch.randn(4, 3, 96, 96, device="cuda").to(torch.bfloat16))
    g = _cl(torch.randn(4, 64, 24, 24, device="cuda", generator=torch.Generator("cuda").manual_seed(2))
            .to(torch.bfloat16))
    res = []
    for path in ("s2d", "direct", "fp32"):
        monkeypatch.setenv("PDT_STEM_S2D", "0" if path == "direct" else "1")
        for p_ in (conv.weight, bn.weight, bn.bias):
            p_.grad = None
        if path == "fp32":
            t = F.conv2d(x.float(), conv.weight, None, 2, 3)
            t = F.relu(F.batch_norm(t, None, None, bn.weight, bn.bias, True, 0.0, bn.eps))
            y = F.max_pool2d(t, 3, 2, 1)
        else:
            no._S2D_W.clear()
            y = no.stem_pool(x, conv, bn)
            assert (id(conv.weight) in no._S2D_W) == (path == "s2d")  # the path under test ran
        y.backward(g.to(y.dtype))
        torch.cuda.synchronize()
        res.append((y.float(), conv.weight.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone()))
    s2d, direct, ref = res
    assert s2d[0].shape == (4, 64, 24, 24)
    for k in range(4):
        es, ed = nrmerr(s2d[k], ref[k]), nrmerr(direct[k], ref[k])
        print(f"stem s2d vs direct {k}: s2d {es:.4g} direct {ed:.4g}")
        assert es < 1.25 * ed + 5e-3, (k, es, ed)


def test_stem_bn_backward_gathers_pool_gradient(monkeypatch):
    """Stem backward with the BN-backward passes gathering dA from the max-pool
    gradient + argmax (no full-resolution dA) vs the maxpool_bwd + BN-backward
    composition (PDT_STEM_POOL_BWD_FUSED=0, the default): the same math except that the
    composition rounds dA to bf16, so the two agree to bf16 rounding."""
    torch.manual_seed(11)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda().to(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(64).cuda()
    with torch.no_grad():
        bn.weight.uniform_(-1.0, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    x = _cl(torch.randn(6, 3, 80, 80, device="cuda").to(torch.bfloat16))
    g = _cl(torch.randn(6, 64, 20, 20, device="cuda", generator=torch.Generator("cuda").manual_seed(4))
            .to(torch.bfloat16))
    res = []
    for fused in ("1", "0"):
        monkeypatch.setenv("PDT_STEM_POOL_BWD_FUSED", fused)
        for p_ in (conv.weight, bn.weight, bn.bias):
            p_.grad = None
        y = no.stem_pool(x, conv, bn)
        y.backward(g)
        torch.cuda.synchronize()
        res.append((conv.weight.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone()))
    for a, b in zip(*res):
        e = nrmerr(a, b)
        print(f"pool-gather vs composed {tuple(a.shape)}: {e:.3g}")
        assert torch.isfinite(a).all() and e < 1e-2, (a.shape, e)


@pytest.mark.parametrize("ncol,use_mask,use_add,use_amask,two", [
    (128, False, True, True, False), (512, True, False, False, False),  # run-time flags (generic walk)
    (256, False, False, False, False),                 # a block's inner unit: ReLU gate from y
    (256, True, True, True, False), (384, True, True, False, False),  # block input: addend, ReLU bits
    (256, True, True, True, True), (384, True, True, False, True)])   # + a second unit's partials
def test_bnb_epilogue_every_variant(ncol, use_mask, use_add, use_amask, two):
    """Every conv_nt tile variant (and stream variant) with the fused BN-backward
    epilogue, on a 1x1 data-gradient geometry: the output (+ ReLU-masked addend)
    and the partial sums (sum of the gated gradient g, sum of g * (y - mean)) vs
    an fp32 reference. The configurations cover the epilogue's compiled walks
    (csrc/conv_nt_tile.inc) and its run-time-flag one."""
    torch.manual_seed(21)
    dev = "cuda"
    N, H, K = 4, 28, 256
    M = N * H * H
    lib = no._load()
    dy = torch.randn(M, K, device=dev).to(torch.bfloat16)
    wt = (torch.randn(ncol, K, device=dev) / K ** 0.5).to(torch.bfloat16)  # B: [Ncol][K]
    y = torch.randn(M, ncol, device=dev).to(torch.bfloat16)
    mean = torch.randn(ncol, device=dev) * 0.1
    scale = torch.rand(ncol, device=dev) + 0.5
    shift = torch.randn(ncol, device=dev) * 0.2
    add = torch.randn(M, ncol, device=dev).to(torch.bfloat16) if use_add else None
    amask = torch.randint(0, 256, (M * ncol // 8,), dtype=torch.uint8, device=dev) if use_amask else None
    mask = torch.randint(0, 256, (M * ncol // 8,), dtype=torch.uint8, device=dev) if use_mask else None

    y2 = torch.randn(M, ncol, device=dev).to(torch.bfloat16) if two else None
    mean2 = torch.randn(ncol, device=dev) * 0.1 if two else None

    def bits(m):
        return ((m.view(-1, 1).int() >> torch.arange(8, device=dev)) & 1).view(M, ncol).float()

    ref = dy.float() @ wt.float().t()
    if use_add:
        ref = ref + add.float() * (bits(amask) if use_amask else 1.0)
    gate = bits(mask) if use_mask else ((y.float() * scale + shift) > 0).float()
    ran = 0
    for v in range(lib.pdt_conv_nt_num_variants()):
        R = lib.pdt_conv_nt_bnb_rows(M, ncol, K, v)
        part = torch.full((2 * max(R, 1) * ncol,), float("nan"), device=dev)
        part2 = torch.full_like(part, float("nan")) if two else None
        out = torch.empty(M, ncol, device=dev, dtype=torch.bfloat16)
        args = (no._p(dy), no._p(wt), no._p(out), no._p(add), no._p(amask), H, H, K, N, H, H, ncol, K, K, 1, 1, 0,
                0, 1, 1, 1, 1, H, H, 1, 1, 0, 0, ncol, v, no._p(y), no._p(mean), no._p(scale), no._p(shift),
                no._p(mask), no._p(part), 1, 0, R)
        if two:
            rc = lib.pdt_conv_nt_bnb2(*args, no._p(y2), no._p(mean2), no._p(part2), no._s())
        else:
            rc = lib.pdt_conv_nt_bnb(*args, no._s())
        if rc == no.NOT_APPLICABLE:
            continue
        assert rc == 0, (v, rc)
        ran += 1
        assert nrmerr(out, ref) < 1e-2, v
        g = out.float() * gate  # the partials see the stored bf16 value
        ps = part.view(2, R, ncol).sum(1)
        assert nrmerr(ps[0], g.sum(0)) < 1e-3, v
        assert nrmerr(ps[1], (g * (y.float() - mean)).sum(0)) < 1e-3, v
        if two:
            ps2 = part2.view(2, R, ncol).sum(1)
            assert torch.equal(ps2[0], ps[0]), v
            assert nrmerr(ps2[1], (g * (y2.float() - mean2)).sum(0)) < 1e-3, v
    # the ring tiles (ids 34-37, persistent 45-46) take only the inner / block-input walks
    compiled = (not use_add and not use_mask) or (use_add and use_mask)
    print(f"variants run: {ran}")
    assert ran >= (30 if compiled and not two else 20)

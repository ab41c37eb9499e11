"""Fusions of the native ViT path against plain PyTorch fp32 references:

* nn.Linear bias gradient computed inside the weight-gradient kernel (every tile variant)
* GELU backward in the data-gradient GEMM epilogue (conv_nt act 3, bf16 and fp8)
* residual add in the linear GEMM epilogue (bf16 and fp8) and its gradient
* LayerNorm fork: residual gradient summed inside the LayerNorm backward
* the fused transformer MLP node, and a 2-block ViT vs the torch path in fp32
* fp8: LayerNorm forward emitting the next GEMM's e4m3 input (bit-exact vs the separate
  delayed-scaling cast), and a 2-block fp8 ViT over several steps (delayed scaling for
  activations and e5m2 output gradients) vs the torch path in fp32
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from pytorch_distributed_template_amd.ops import fused  # noqa: E402
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def nrmerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


def setup_module(module):
    assert no.available(), "native library must be built and loaded on GPU runs"
    no.require()


def _gelu_grad(z):
    u = 0.7978845608 * (z + 0.044715 * z ** 3)
    t = torch.tanh(u)
    return 0.5 * (1 + t) + 0.5 * z * (1 - t * t) * 0.7978845608 * (1 + 3 * 0.044715 * z * z)


@pytest.mark.parametrize("M,Nout,K", [(1576, 768, 2304), (600, 256, 128), (4096, 3072, 768)])
def test_wgrad_fused_bias_all_variants(M, Nout, K):
    torch.manual_seed(M + Nout)
    dy = torch.randn(M, Nout, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    ref_w = dy.float().t() @ x.float()
    ref_b = dy.float().sum(0)
    lib = no._load()
    for v in range(lib.pdt_wgrad_num_variants()):
        dw = torch.empty(Nout, K, device="cuda")
        db = torch.full((Nout,), float("nan"), device="cuda")
        no.conv_wgrad(dy, x, dw, M=M, Mo=Nout, No=K, ldy=Nout, Hs=1, Ws=1, C=K, Hm=1, Wm=1, sh=1, sw=1, oh0=0, ow0=0,
                      dh=1, dw=1, ntw=1, variant=v, bias_out=db)
        torch.cuda.synchronize()
        assert nrmerr(dw, ref_w) < 1e-2, (v, nrmerr(dw, ref_w))
        assert nrmerr(db, ref_b) < 1e-5, (v, nrmerr(db, ref_b))


def test_gelu_backward_epilogue_bf16_and_fp8():
    torch.manual_seed(21)
    M, N, K = 1000, 3072, 768          # dz[M, N] = (g[M, K] @ W[K, N]) * gelu'(z)
    g = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(K, N, device="cuda") * 0.05          # fc2 weight [Nout=K][K=N]
    z = (torch.randn(M, N, device="cuda") * 2).to(torch.bfloat16)
    ref = (g.float() @ w.to(torch.bfloat16).float()) * _gelu_grad(z.float())
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    no._gemm_bf16(g, no.bf16_weight_t(w), out, act=3, addend=z)
    torch.cuda.synchronize()
    assert nrmerr(out, ref) < 1e-2, nrmerr(out, ref)
    gq, dqg = no.quantize_fp8(g, no.E5M2)
    _, wqt, dqw = no.fp8_weight(w)
    ref8 = ((gq.view(torch.float8_e5m2).float() * dqg) @ (wqt.view(torch.float8_e4m3fn).float() * dqw).t()) \
        * _gelu_grad(z.float())
    out8 = torch.empty_like(out)
    no.gemm_f8(gq, wqt, out8, dqg, dqw, fmt_a=no.E5M2, act=3, addend=z)
    torch.cuda.synchronize()
    assert nrmerr(out8, ref8) < 1e-2, nrmerr(out8, ref8)


@pytest.mark.parametrize("fp8", [False, True])
def test_linear_residual_epilogue(fp8):
    torch.manual_seed(22)
    fc = nn.Linear(768, 768).cuda()
    x = torch.randn(3, 197, 768, device="cuda").to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(3, 197, 768, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = no.linear(x, fc, fp8=fp8, residual=r)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True)
    wr = fc.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.linear(xr, wr, fc.bias.detach()) + rr
    assert nrmerr(y, yr) < (4e-2 if fp8 else 1e-2), nrmerr(y, yr)
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    assert torch.equal(r.grad, g)  # the residual gradient is dy itself
    # fp8: the data and weight gradients run on e5m2 output gradients (2 mantissa bits)
    assert nrmerr(x.grad, xr.grad) < (8e-2 if fp8 else 2e-2), nrmerr(x.grad, xr.grad)
    assert nrmerr(fc.weight.grad, wr.grad) < (8e-2 if fp8 else 2e-2), nrmerr(fc.weight.grad, wr.grad)
    assert nrmerr(fc.bias.grad, g.float().sum((0, 1))) < 1e-4


def test_ln_fork_sums_residual_gradient():
    torch.manual_seed(23)
    ln = nn.LayerNorm(768, eps=1e-6).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    x = torch.randn(2, 197, 768, device="cuda").to(torch.bfloat16).requires_grad_(True)
    xid, h = no.ln_fork(x, ln)
    xr = x.detach().float().requires_grad_(True)
    hr = F.layer_norm(xr, (768,), ln.weight, ln.bias, 1e-6)
    assert nrmerr(h, hr) < 1e-2
    gh = torch.randn_like(hr).to(torch.bfloat16)
    gres = torch.randn_like(hr).to(torch.bfloat16)
    ((xid.float() * gres.float()).sum() + (h.float() * gh.float()).sum()).backward()
    ((xr * gres.float()).sum() + (hr * gh.float()).sum()).backward()
    assert nrmerr(x.grad, xr.grad) < 2e-2, nrmerr(x.grad, xr.grad)


@pytest.mark.parametrize("M,Nout,K", [(600, 256, 128), (1576, 2304, 768), (4096, 768, 3072)])
def test_linear_wgrad_f8_all_variants(M, Nout, K):
    """fp8 weight gradient (csrc/wgrad_f8.hip, ds_read_b64_tr_b8 + 16x16x128 f8f6f4 MFMA) ==
    the fp32 product of the dequantised e5m2 dY / e4m3 X codes, every tile variant; bias
    gradient == column sums of the bf16 dY. M % 128 != 0 exercises the zero-filled tail."""
    torch.manual_seed(M + K)
    dy = torch.randn(M, Nout, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    dyq, dqdy = no.quantize_fp8(dy, no.E5M2)
    xq, dqx = no.quantize_fp8(x, no.E4M3)
    ref = (dyq.view(torch.float8_e5m2).float() * dqdy).t() @ (xq.view(torch.float8_e4m3fn).float() * dqx)
    lib = no._load()
    for v in range(lib.pdt_wgrad_f8_num_variants()):
        dw, db = no.linear_wgrad_f8(dyq, xq, dqdy, dqx, dy16=dy, with_bias=True, variant=v)
        e = nrmerr(dw, ref)
        assert e < 1e-4, (v, e)  # fp32 summation order / dequant placement only
        assert nrmerr(db, dy.float().sum(0)) < 1e-5, v
    # and the quantisation budget vs the exact bf16 operands (e5m2 keeps 2 mantissa bits)
    exact = dy.float().t() @ x.float()
    assert nrmerr(dw, exact) < 0.1, nrmerr(dw, exact)


@pytest.mark.parametrize("act,qfmt", [(2, 0), (3, 1), (0, 0)])
def test_gemm_f8_fp8_output_epilogue(act, qfmt):
    """gemm_f8(q8=...): the epilogue's fp8 codes, dequant factor and amax-history roll equal
    the bf16 output followed by the separate delayed-scaling cast, for every variant that
    supports it (GELU forward -> e4m3, GELU backward -> e5m2, plain)."""
    torch.manual_seed(40 + act)
    M, N, K = 1000, 384, 256
    a8, dqa = no.quantize_fp8(torch.randn(M, K, device="cuda").to(torch.bfloat16), no.E4M3 if act != 3 else no.E5M2)
    b8, dqb = no.quantize_fp8(torch.randn(N, K, device="cuda").to(torch.bfloat16) * 0.1, no.E4M3)
    fmt_a = no.E5M2 if act == 3 else no.E4M3
    z = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    bias = torch.randn(N, device="cuda") if act == 2 else None
    kw = dict(fmt_a=fmt_a, bias=bias, act=act, addend=z if act == 3 else None,
              aux=torch.empty(M, N, dtype=torch.bfloat16, device="cuda") if act == 2 else None)
    _, _, meta0 = no.quantize_fp8_delayed(torch.randn(M, N, device="cuda").to(torch.bfloat16), None, qfmt)
    lib = no._load()
    for v in range(lib.pdt_gemm_f8_num_variants()):
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        try:
            no.gemm_f8(a8, b8, out, dqa, dqb, variant=v, **kw)
        except no.NotApplicable:  # (the dense ring: plain epilogue, N % 256 == 0)
            continue
        q_ref, dq_ref, meta_ref = no.quantize_fp8_delayed(out, meta0.clone(), qfmt)
        out2 = torch.empty_like(out)
        codes = torch.empty(M, N, dtype=torch.uint8, device="cuda")
        meta = meta0.clone()
        part = torch.empty(lib.pdt_gemm_f8_q8_part(M, N) + 1, device="cuda")
        args = (no._p(a8), no._p(b8), no._p(out2), no._p(bias), no._p(dqa), no._p(dqb), M, N, K, K, K, N, fmt_a, act,
                no._p(kw["aux"]), no._p(kw["addend"]), v, no._p(codes), no._p(meta), no._p(part), qfmt, 0,
                no._p(part[-1:]), no._s())
        rc = lib.pdt_gemm_f8_q8(*args)
        if rc == no.NOT_APPLICABLE:
            continue
        assert rc == 0, (v, rc)
        torch.cuda.synchronize()
        assert torch.equal(out2, out), v
        assert torch.equal(codes, q_ref), (v, (codes != q_ref).sum().item())
        assert torch.equal(part[-1:], dq_ref), v
        assert torch.equal(meta, meta_ref), v


def test_ln_fork_fp8_codes_match_separate_cast(monkeypatch):
    """pdt_ln_fwd_f8: same e4m3 codes, dq and amax-history roll as LayerNorm followed by
    the delayed-scaling cast (rows % 4 != 0 exercises the idle-wave path); the codes-only
    output (no bf16 values written) carries the same codes."""
    monkeypatch.setenv("PDT_LN_CODES_ONLY", "0")  # the bf16 output is compared below
    torch.manual_seed(26)
    ln = nn.LayerNorm(768, eps=1e-6).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    fc = nn.Linear(768, 256).cuda()
    x = (torch.randn(2, 197, 768, device="cuda") * 2).to(torch.bfloat16)
    no._quant_act(torch.randn(394, 768, device="cuda").to(torch.bfloat16), fc)  # seed fc's history
    meta0 = fc._pdt_fp8_meta.clone()
    _, h = no.ln_fork(x, ln, fc)
    assert hasattr(h, "_pdt_f8") and h._pdt_f8[2] is fc
    q, dq = h._pdt_f8[0].clone(), h._pdt_f8[1].clone()
    meta1 = fc._pdt_fp8_meta.clone()
    _, h_ref = no.ln_fork(x, ln)
    assert torch.equal(h, h_ref)
    q_ref, dq_ref, meta_ref = no.quantize_fp8_delayed(h_ref.reshape(-1, 768), meta0.clone(), no.E4M3)
    torch.cuda.synchronize()
    assert torch.equal(q.view(-1, 768), q_ref), (q.view(-1, 768) != q_ref).sum().item()
    assert torch.equal(dq, dq_ref)
    assert torch.equal(meta1, meta_ref), (meta1, meta_ref)
    monkeypatch.setenv("PDT_LN_CODES_ONLY", "1")
    fc._pdt_fp8_meta = meta0.clone()
    _, h1 = no.ln_fork(x, ln, fc)
    assert getattr(h1, "_pdt_f8_only", False) and h1._pdt_f8[2] is fc
    assert torch.equal(h1._pdt_f8[0], q) and torch.equal(h1._pdt_f8[1], dq)
    with pytest.raises(RuntimeError, match="codes only"):
        no._prequant(h1, nn.Linear(768, 256).cuda())  # any other consumer would read the values


def test_ln_fork_backward_e5m2_codes_match_separate_cast():
    """pdt_ln_bwd_f8: the e5m2 codes of dx riding on the gradient (for the fp8 layer that
    produced the fork's input) equal the delayed-scaling cast of that gradient."""
    torch.manual_seed(28)
    ln = nn.LayerNorm(768, eps=1e-6).cuda()
    owner = nn.Linear(768, 768).cuda()
    no._quant_grad(torch.randn(394, 768, device="cuda").to(torch.bfloat16), owner, "_pdt_fp8_gmeta")  # seed
    meta0 = owner._pdt_fp8_gmeta.clone()
    captured = []

    class Cap(torch.autograd.Function):
        @staticmethod
        def forward(ctx, t):
            return t.view_as(t)

        @staticmethod
        def backward(ctx, g):
            captured.append(g)
            return g

    x = torch.randn(2, 197, 768, device="cuda").to(torch.bfloat16).requires_grad_(True)
    xid, h = no.ln_fork(Cap.apply(x), ln, grad_fp8_for=owner)
    gh = torch.randn_like(h)
    gres = torch.randn_like(h)
    ((xid.float() * gres.float()).sum() + (h.float() * gh.float()).sum()).backward()
    g = captured[0]
    assert hasattr(g, "_pdt_f8g") and g._pdt_f8g[2] is owner
    q_ref, dq_ref, meta_ref = no.quantize_fp8_delayed(g.reshape(-1, 768), meta0.clone(), no.E5M2)
    torch.cuda.synchronize()
    assert torch.equal(g._pdt_f8g[0].view(-1, 768), q_ref)
    assert torch.equal(g._pdt_f8g[1], dq_ref)
    assert torch.equal(owner._pdt_fp8_gmeta, meta_ref)
    # and the gradient itself is the plain LayerNorm-fork gradient
    x2 = x.detach().clone().requires_grad_(True)
    xid2, h2 = no.ln_fork(x2, ln)
    ((xid2.float() * gres.float()).sum() + (h2.float() * gh.float()).sum()).backward()
    assert torch.equal(x.grad, x2.grad)


def test_attention_fp8_output_codes_match_separate_cast(monkeypatch):
    """pdt_attn_fwd_f8_q8: O unchanged, and the projection's e4m3 input codes / dequant factor /
    amax-history roll equal the delayed-scaling cast of O."""
    torch.manual_seed(29)
    monkeypatch.setenv("PDT_FP8_ATTN_Q8", "1")
    B, T, H = 2, 197, 4
    qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16)
    proj = nn.Linear(H * 64, H * 64).cuda()
    no._quant_act(torch.randn(B * T, H * 64, device="cuda").to(torch.bfloat16), proj)  # seed the history
    meta0 = proj._pdt_fp8_meta.clone()
    o = no.qkv_attention(qkv, H, fp8=True, fp8_for=proj)
    assert hasattr(o, "_pdt_f8") and o._pdt_f8[2] is proj
    codes, dq = o._pdt_f8[0].clone(), o._pdt_f8[1].clone()
    meta1 = proj._pdt_fp8_meta.clone()
    o_ref = no.qkv_attention(qkv, H, fp8=True)
    assert torch.equal(o, o_ref)
    q_ref, dq_ref, meta_ref = no.quantize_fp8_delayed(o_ref.reshape(-1, H * 64), meta0.clone(), no.E4M3)
    torch.cuda.synchronize()
    assert torch.equal(codes, q_ref)
    assert torch.equal(dq, dq_ref)
    assert torch.equal(meta1, meta_ref)


def test_attention_backward_e5m2_codes_match_separate_cast(monkeypatch):
    """pdt_attn_bwd_q8: d(qkv) unchanged, and its e5m2 codes / dequant factor / history roll
    (for the qkv projection) equal the delayed-scaling cast of d(qkv)."""
    torch.manual_seed(30)
    monkeypatch.setenv("PDT_FP8_ATTN_Q8", "1")
    monkeypatch.setenv("PDT_FP8_ATTN_BWD", "0")  # the codes ride on the bf16 backward kernels
    B, T, H = 2, 197, 4
    qkv_fc = nn.Linear(H * 64, 3 * H * 64).cuda()
    no._quant_grad(torch.randn(B * T, 3 * H * 64, device="cuda").to(torch.bfloat16), qkv_fc, "_pdt_fp8_gmeta")
    meta0 = qkv_fc._pdt_fp8_gmeta.clone()
    captured = []

    class Cap(torch.autograd.Function):
        @staticmethod
        def forward(ctx, t):
            return t.view_as(t)

        @staticmethod
        def backward(ctx, g):
            captured.append(g)
            return g

    base = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16)
    gout = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
    x = base.clone().requires_grad_(True)
    no.qkv_attention(Cap.apply(x), H, fp8=True, grad_fp8_for=qkv_fc).backward(gout)
    g = captured[0]
    assert hasattr(g, "_pdt_f8g") and g._pdt_f8g[2] is qkv_fc
    x2 = base.clone().requires_grad_(True)
    no.qkv_attention(x2, H, fp8=True).backward(gout)
    assert torch.equal(x.grad, x2.grad)
    q_ref, dq_ref, meta_ref = no.quantize_fp8_delayed(g.reshape(-1, 3 * H * 64), meta0.clone(), no.E5M2)
    torch.cuda.synchronize()
    assert torch.equal(g._pdt_f8g[0], q_ref)
    assert torch.equal(g._pdt_f8g[1], dq_ref)
    assert torch.equal(qkv_fc._pdt_fp8_gmeta, meta_ref)


def test_vit_fp8_steps_track_torch_fp32():
    """2-block fp8 ViT, three forward/backward passes (the first seeds the delayed-scaling
    histories; the later ones take the LayerNorm-fused e4m3 inputs and delayed e5m2
    gradient scales) vs the torch path in fp32 on the same weights."""
    from pytorch_distributed_template_amd.models.vit import VisionTransformer
    torch.manual_seed(27)
    m = VisionTransformer(depth=2, num_classes=32, fp8=True).cuda()
    x = torch.randn(4, 3, 224, 224, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 32, (4,), device="cuda")
    errs = []
    for it in range(3):
        out = {}
        for backend in ("native", "torch"):
            fused.set_backend(backend)
            m.zero_grad(set_to_none=True)
            logits = m(x if backend == "native" else x.float())
            fused.softmax_cross_entropy(logits, t).backward()
            out[backend] = (logits.detach().float(), {n: p.grad.detach().float().clone()
                                                      for n, p in m.named_parameters()})
        fused.set_backend("auto")
        el = nrmerr(out["native"][0], out["torch"][0])
        worst = max((nrmerr(out["native"][1][n], out["torch"][1][n]), n) for n in out["torch"][1])
        errs.append((it, el, worst))
    print(errs)
    # 128 logits of a random-init model: the fp8 quantisation noise realised in them moves with
    # bit-level rounding of the bf16 inputs (0.073 with the implicit-GEMM patch embedding, 0.083
    # with patchify + GEMM, whose tokens are as accurate: scripts/probe_patch_embed.py)
    for it, el, worst in errs:
        assert el < 0.1, errs
        assert worst[0] < 0.25, errs
    assert m.blocks[0].attn.qkv._pdt_fp8_meta is not None and m.blocks[0].mlp.fc2._pdt_fp8_gmeta is not None


@pytest.mark.parametrize("mode", ["bf16", "fp8", "fp8_lib", "fp8_lib_natdgrad", "fp8_lib_aux", "bf16_nodual",
                                  "fp8_nodual"])
def test_fused_mlp_node(mode, monkeypatch):
    """The MLP node vs fp32 autograd. fp8: delayed scaling, so a first step seeds the amax
    histories and the checked step runs the fused fc1 epilogue (act 4 + e4m3 side output);
    fp8_lib: fc1 on the library GEMM + pdt_gelu_dual_cast_fp8 keeping the GEMM's pre-activation
    (the fc2 data gradient forms gelu'(z), act 3); fp8_lib_aux: the cast pass writes gelu'(z)
    (act 5); fp8_lib runs the fc2 data gradient on the library GEMM + the gelu'-multiplying e5m2
    cast with bias sums, fp8_lib_natdgrad on the native tile's act-3 epilogue; *_nodual: z
    stored, gelu'(z) recomputed in the fc2 data-gradient epilogue (acts 2 / 3)."""
    from pytorch_distributed_template_amd.models.vit import Mlp
    fp8 = mode.startswith("fp8")
    monkeypatch.setenv("PDT_GELU_DUAL", "0" if mode.endswith("nodual") else "1")
    monkeypatch.setenv("PDT_FP8_FC1_LIB", "1" if mode.startswith("fp8_lib") else "0")
    monkeypatch.setenv("PDT_FC1_KEEP_PRE", "0" if mode == "fp8_lib_aux" else "1")
    monkeypatch.setenv("PDT_FC2_DGRAD_LIB", "0" if mode == "fp8_lib_natdgrad" else "1")
    torch.manual_seed(24)
    m = Mlp(768, 3072).cuda()
    x = torch.randn(4, 197, 768, device="cuda").to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(4, 197, 768, device="cuda").to(torch.bfloat16).requires_grad_(True)
    g = torch.randn(4, 197, 768, device="cuda").to(torch.bfloat16)
    # a first step seeds the fp8 amax histories (with the gradient of the checked step: a
    # delayed scale from another distribution would saturate the e5m2 codes)
    no.mlp(x, m, fp8=fp8, residual=r).backward(g)
    for t in (x, r, m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias):
        t.grad = None
    y = no.mlp(x, m, fp8=fp8, residual=r)
    assert "Mlp" in type(y.grad_fn).__name__
    xr = x.detach().float().requires_grad_(True)
    w1 = m.fc1.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    w2 = m.fc2.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    b1 = m.fc1.bias.detach().clone().requires_grad_(True)
    b2 = m.fc2.bias.detach().clone().requires_grad_(True)
    yr = F.linear(F.gelu(F.linear(xr, w1, b1), approximate="tanh"), w2, b2) + r.detach().float()
    tol = 6e-2 if fp8 else 1.5e-2
    assert nrmerr(y, yr) < tol, nrmerr(y, yr)
    y.backward(g)
    yr.backward(g.float())
    assert torch.equal(r.grad, g)
    for got, ref, name in ((x.grad, xr.grad, "dx"), (m.fc1.weight.grad, w1.grad, "dw1"),
                           (m.fc2.weight.grad, w2.grad, "dw2"), (m.fc1.bias.grad, b1.grad, "db1"),
                           (m.fc2.bias.grad, b2.grad, "db2")):
        e = nrmerr(got, ref)
        assert e < (1e-1 if fp8 else 3e-2), (name, e)


def test_vit_native_matches_torch_fp32():
    """2-block ViT-B/16: native bf16 forward/backward vs the torch path in fp32 (same weights)."""
    from pytorch_distributed_template_amd.models.vit import VisionTransformer
    torch.manual_seed(25)
    m = VisionTransformer(depth=2, num_classes=32).cuda()
    x = torch.randn(4, 3, 224, 224, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 32, (4,), device="cuda")
    out = {}
    for backend in ("native", "torch"):
        fused.set_backend(backend)
        m.zero_grad(set_to_none=True)
        logits = m(x if backend == "native" else x.float())
        loss = fused.softmax_cross_entropy(logits, t)
        loss.backward()
        out[backend] = (logits.detach().float(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()})
    fused.set_backend("auto")
    assert nrmerr(out["native"][0], out["torch"][0]) < 3e-2
    worst = max((nrmerr(out["native"][1][n], out["torch"][1][n]), n) for n in out["torch"][1])
    assert worst[0] < 8e-2, worst


def _pow2_scale(amax):
    e = torch.floor(torch.log2(448.0 / amax.clamp_min(1e-30)))
    return torch.where(amax > 0, torch.exp2(e.clamp(-100, 100)), torch.ones_like(amax))


def _fp8_emulated_scores(q, k):
    """S = Q K^T with Q, K quantized exactly as csrc/attention_f8.hip does: K per (b, h)
    and Q per (b, h, 32-query tile) with power-of-two scales, e4m3 round-to-nearest."""
    B, H, T, _ = q.shape
    sk = _pow2_scale(k.abs().amax(dim=(2, 3), keepdim=True))
    kq = (k * sk).to(torch.float8_e4m3fn).float() / sk
    nqt = (T + 31) // 32
    qp = torch.nn.functional.pad(q, (0, 0, 0, nqt * 32 - T)).view(B, H, nqt, 32, 64)
    sq = _pow2_scale(qp.abs().amax(dim=(3, 4), keepdim=True))
    qq = ((qp * sq).to(torch.float8_e4m3fn).float() / sq).view(B, H, nqt * 32, 64)[:, :, :T]
    return qq @ kq.transpose(-1, -2)


def _fp8_emulated_pv(s8, v):
    """O = softmax(S) V as csrc/attention_f8.hip computes it on fp8: keys in pairs of 32-key
    tiles, running max / rescale per pair, P coded as e4m3(256 exp2(S log2e - m_running)),
    V per (b, h) power-of-two e4m3, row sums of the fp32 P."""
    B, H, T, _ = s8.shape
    sv = _pow2_scale(v.abs().amax(dim=(2, 3), keepdim=True))
    vq = (v * sv).to(torch.float8_e4m3fn).float() / sv
    z = s8 / 0.6931471805599453  # log2 domain
    m = torch.full((B, H, T, 1), -float("inf"), device=s8.device)
    l = torch.zeros((B, H, T, 1), device=s8.device)
    o = torch.zeros((B, H, T, 64), device=s8.device)
    for k0 in range(0, T, 64):
        zs = z[..., k0:k0 + 64]
        mn = torch.maximum(m, zs.amax(-1, keepdim=True))
        alpha = torch.exp2(m - mn)
        p = torch.exp2(zs - mn)
        p8 = (p * 256).to(torch.float8_e4m3fn).float() / 256
        o = o * alpha + p8 @ vq[:, :, k0:k0 + 64]
        l = l * alpha + p.sum(-1, keepdim=True)
        m = mn
    return o / l


@pytest.mark.parametrize("bwd,pv8", [("f8", False), ("bf16", False), ("f8", True)])
@pytest.mark.parametrize("B,T,H", [(3, 197, 4), (2, 64, 2), (1, 50, 12), (2, 256, 3), (2, 16, 3), (1, 120, 2)])
def test_fp8_attention_forward_and_backward(B, T, H, bwd, pv8, monkeypatch):
    """fp8 attention forward (csrc/attention_f8.hip: e4m3 S = Q K^T and O = P V): (1) against
    a reference that applies the kernel's own quantization (per-head K / V and per-32-query-
    tile Q power-of-two scales, P coded per key-tile pair, e4m3) in fp32 -- checks the kernel
    itself tightly; (2) against exact fp32 attention -- the
    fp8 error budget, with the fused fp8 backward (csrc/attention_bwd_f8.hip, the default
    for fp8 attention) or the bf16 recomputing one run on its output and LSE. ``pv8``: the
    PV GEMM on e4m3 too (PDT_FP8_ATTN_PV=1; default bf16 PV)."""
    monkeypatch.setenv("PDT_FP8_ATTN_BWD", "1" if bwd == "f8" else "0")
    no._load().pdt_attn_set_pv8(int(pv8))
    torch.manual_seed(B * 100 + T)
    qkv = (torch.randn(B, T, 3 * H * 64, device="cuda") * 1.5).to(torch.bfloat16)
    dout = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
    x = qkv.float().requires_grad_(True)
    q, k, v = x.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / 8.0
    ref = (torch.softmax(s, dim=-1) @ v).transpose(1, 2).reshape(B, T, H * 64)
    ref.backward(dout.float())
    with torch.no_grad():
        s8 = _fp8_emulated_scores(q.detach(), k.detach()) / 8.0
        if pv8:
            ref8 = _fp8_emulated_pv(s8, v.detach()).transpose(1, 2).reshape(B, T, H * 64)
        else:
            ref8 = (torch.softmax(s8, dim=-1) @ v.detach()).transpose(1, 2).reshape(B, T, H * 64)
        lse8 = torch.logsumexp(s8, dim=-1) / 0.6931471805599453  # log2 domain
    xn = qkv.clone().requires_grad_(True)
    try:
        out = no.qkv_attention(xn, H, fp8=True)
    finally:
        no._load().pdt_attn_set_pv8(0)
    lse = out.grad_fn.saved_tensors[2].view(B, H, T)
    e8 = nrmerr(out, ref8)
    dl = (lse - lse8).abs().max().item()
    assert e8 < 1e-2 and dl < 5e-2, (e8, dl)  # the kernel == its quantization model
    out.backward(dout)
    torch.cuda.synchronize()
    assert out.shape == ref.shape and out.dtype == torch.bfloat16
    e = nrmerr(out, ref)
    # fp8 error budget vs exact attention (x1.5 inputs; the score GEMM's e4m3 error dominates:
    # 0.065 at T=197 with bf16 PV, round 2)
    assert e < 9e-2, e
    g, gr = xn.grad.view(B, T, 3, H * 64), x.grad.view(B, T, 3, H * 64)
    for i, name in enumerate("qkv"):
        ei = nrmerr(g[:, :, i], gr[:, :, i])
        # fp8 backward: its own e4m3 score recompute adds ~0.1 (tests/test_attention_bwd_f8_gpu.py)
        assert ei < (1.6e-1 if bwd == "f8" else 1e-1), (name, ei)


@pytest.mark.parametrize("fp8,codes_only", [(False, "0"), (True, "0"), (True, "1")])
def test_ln_add_fork_matches_add_then_fork(fp8, codes_only, monkeypatch):
    """ln_add_fork(y, r) == ln_fork(bf16(y + r)): the summed residual stream, the normalised
    output (and its e4m3 codes under delayed scaling), and both input gradients = the fork's
    summed gradient (with the producer's e5m2 codes). codes_only: the normalised output is
    written as e4m3 codes alone (its values are then not compared)."""
    monkeypatch.setenv("PDT_LN_CODES_ONLY", codes_only)
    torch.manual_seed(41)
    D, rows = 768, 394
    ln = nn.LayerNorm(D, eps=1e-6).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    consumer, producer = nn.Linear(D, D).cuda(), nn.Linear(D, D).cuda()
    if fp8:
        no._quant_act(torch.randn(rows, D, device="cuda").to(torch.bfloat16), consumer)
        no._quant_grad(torch.randn(rows, D, device="cuda").to(torch.bfloat16), producer, "_pdt_fp8_gmeta")
    y0 = torch.randn(2, rows // 2, D, device="cuda").to(torch.bfloat16)
    r0 = torch.randn(2, rows // 2, D, device="cuda").to(torch.bfloat16)
    g_res = torch.randn_like(y0)
    g_h = torch.randn_like(y0)
    metas = [(getattr(consumer, "_pdt_fp8_meta", None), getattr(producer, "_pdt_fp8_gmeta", None))]

    def run(fused_add):
        if fp8:  # both runs start from the same scaling state
            consumer._pdt_fp8_meta = metas[0][0].clone()
            producer._pdt_fp8_gmeta = metas[0][1].clone()
        y = y0.clone().requires_grad_(True)
        r = r0.clone().requires_grad_(True)
        cons, prod = (consumer, producer) if fp8 else (None, None)
        if fused_add:
            s, h = no.ln_add_fork(y, r, ln, cons, prod)
        else:
            s, h = no.ln_fork(y + r, ln, cons, prod)
        torch.autograd.backward([s, h], [g_res, g_h])
        return s, h, y.grad, r.grad

    s1, h1, gy1, gr1 = run(True)
    s0, h0, gy0, gr0 = run(False)
    torch.cuda.synchronize()
    assert torch.equal(s1, s0)
    if codes_only == "1":
        assert getattr(h1, "_pdt_f8_only", False) and getattr(h0, "_pdt_f8_only", False)
    else:
        assert torch.equal(h1, h0)
    assert torch.equal(gy1, gy0) and torch.equal(gr1, gy1)
    if fp8:
        assert torch.equal(h1._pdt_f8[0], h0._pdt_f8[0])
        assert torch.equal(gy1._pdt_f8g[0], gy0._pdt_f8g[0]) if hasattr(gy0, "_pdt_f8g") else True


def test_ln_backward_bias_grads_match_wgrad_bias(monkeypatch):
    """Bias gradients formed where the gradient is written -- proj / fc2 in the LayerNorm
    backward (PDT_LN_DB), fc1 in the fc2 data-gradient epilogue (PDT_F8_DB_EPI), qkv in the
    e5m2 cast of its output gradient (PDT_CAST_DB) -- equal the ones the fp8 weight-gradient
    kernel sums from the same bf16 gradients (2-block fp8 ViT, second step so the
    delayed-scaling state exists)."""
    from pytorch_distributed_template_amd.models import vit_b_16
    grads = {}
    for mode in ("0", "1"):
        for var in ("PDT_LN_DB", "PDT_F8_DB_EPI", "PDT_CAST_DB"):
            monkeypatch.setenv(var, mode)
        torch.manual_seed(51)
        m = vit_b_16(num_classes=16, fp8=True, depth=2).cuda()
        x = torch.randn(4, 3, 224, 224, device="cuda")
        for _ in range(2):
            m.zero_grad(set_to_none=True)
            m(x).float().square().mean().backward()
        torch.cuda.synchronize()
        grads[mode] = {n: p.grad.detach().clone() for n, p in m.named_parameters()
                       if n.endswith("bias") and any(k in n for k in ("qkv", "proj", "fc1", "fc2"))}
    assert grads["1"].keys() == grads["0"].keys() and len(grads["1"]) == 8
    for n in grads["1"]:
        assert nrmerr(grads["1"][n], grads["0"][n]) < 1e-3, n


@pytest.mark.parametrize("variant", [8, 9, 10])
def test_gemm_f8_epilogue_column_sums(variant):
    """gemm_f8(..., q8=(codes, meta, fmt, only=True), colsum_out=...): the column sums of the
    final bf16 output (act 5: out * addend) formed in the epilogue equal the sums of the output
    a plain call writes, and the codes / dequant factor are the same."""
    torch.manual_seed(61)
    M, N, K = 1000, 768, 256
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda")
    qa, dqa = no.quantize_fp8(a, no.E5M2)
    qb, dqb = no.quantize_fp8(b, no.E4M3)
    add = torch.rand(M, N, device="cuda").to(torch.bfloat16)
    meta = no.quantize_fp8_delayed(torch.randn(M, N, device="cuda").to(torch.bfloat16), None, no.E5M2)[2]
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    codes = torch.empty(M, N, device="cuda", dtype=torch.uint8)
    m0 = meta.clone()
    dq0 = no.gemm_f8(qa, qb, out, dqa, dqb, fmt_a=no.E5M2, act=no.ACT_MUL, addend=add, variant=variant,
                     q8=(codes, m0, no.E5M2, False))
    cs = torch.full((N,), float("nan"), device="cuda")
    codes1 = torch.empty_like(codes)
    m1 = meta.clone()
    out1 = torch.full_like(out, float("nan"))
    dq1 = no.gemm_f8(qa, qb, out1, dqa, dqb, fmt_a=no.E5M2, act=no.ACT_MUL, addend=add, variant=variant,
                     q8=(codes1, m1, no.E5M2, True), colsum_out=cs)
    torch.cuda.synchronize()
    assert torch.isnan(out1.float()).all()  # q8 only: the bf16 output is not written
    assert torch.equal(codes1, codes) and torch.equal(dq1, dq0) and torch.equal(m1, m0)
    ref = out.float().sum(0)
    assert nrmerr(cs, ref) < 1e-5, nrmerr(cs, ref)


@pytest.mark.parametrize("layout", ["channels_last", "contiguous"])
@pytest.mark.parametrize("path", ["linear", "implicit"])
def test_patch_embedding_matches_conv_fp32(layout, path, monkeypatch):
    """Patch embedding (patchify + plain GEMM, or the channel-padded implicit GEMM) vs an fp32
    conv: tokens, weight gradient and bias gradient, for both weight memory layouts."""
    monkeypatch.setenv("PDT_PATCH_LINEAR", "1" if path == "linear" else "0")
    torch.manual_seed(0)
    conv = nn.Conv2d(3, 768, 16, stride=16).cuda()
    mf = torch.channels_last if layout == "channels_last" else torch.contiguous_format
    conv = conv.to(memory_format=mf)
    x = torch.randn(4, 3, 224, 224, device="cuda").to(torch.bfloat16)
    g = torch.randn(4, 196, 768, device="cuda")
    ref = nn.Conv2d(3, 768, 16, stride=16).cuda()
    ref.load_state_dict(conv.state_dict())
    yr = ref(x.float()).flatten(2).transpose(1, 2)
    yr.backward(g)
    y = no.patch_embed(x, conv)
    y.backward(g.to(torch.bfloat16))
    assert y.shape == (4, 196, 768)
    assert nrmerr(y, yr) < 1e-2
    assert conv.weight.grad.shape == ref.weight.grad.shape
    assert nrmerr(conv.weight.grad, ref.weight.grad) < 1e-2
    assert nrmerr(conv.bias.grad, ref.bias.grad) < 1e-2


def test_embed_tokens_matches_cat_add():
    """Token assembly ([cls; tok] + pos in one pass) vs torch.cat + add in fp32: values and
    the gradients of the tokens, the class token and the position embedding."""
    torch.manual_seed(0)
    B, N, D = 6, 196, 768
    tok = torch.randn(B, N, D, device="cuda").to(torch.bfloat16).requires_grad_()
    cls = (0.02 * torch.randn(1, 1, D, device="cuda")).requires_grad_()
    pos = (0.02 * torch.randn(1, N + 1, D, device="cuda")).requires_grad_()
    g = torch.randn(B, N + 1, D, device="cuda")
    x = no.embed_tokens(tok, cls, pos)
    gt, gc, gp = torch.autograd.grad(x, (tok, cls, pos), g.to(torch.bfloat16))
    t32 = tok.detach().float().requires_grad_()
    xr = torch.cat([cls.expand(B, -1, -1), t32], dim=1) + pos
    rt, rc, rp = torch.autograd.grad(xr, (t32, cls, pos), g)
    assert x.shape == (B, N + 1, D) and x.dtype == torch.bfloat16
    assert nrmerr(x, xr) < 5e-3
    assert nrmerr(gt, rt) < 5e-3 and nrmerr(gc, rc) < 5e-3 and nrmerr(gp, rp) < 5e-3
    assert gc.shape == cls.shape and gp.shape == pos.shape


@pytest.mark.parametrize("act,qfmt,cs", [(4, 0, False), (3, 1, True), (5, 1, True), (0, 0, False)])
def test_ring_fused_epilogues(act, qfmt, cs):
    """The dense 256x256 ring (fp8 variant 12, csrc/gemm_ring.hip) with the fused epilogues of
    the ViT MLP: fc1's GELU + gelu' (act 4) with fc2's e4m3 input codes, the fc2 data gradient's
    gelu' multiply (act 3 / 5) with fc1's e5m2 gradient codes and bias-gradient column sums, a
    residual addend (act 0): the bf16 output against the staged native tile (variant 1), the
    codes / dequant factor / amax history against the separate cast of the ring's own output
    (bit-exact), the column sums against a sum of that output; M has a partial 256-row tile."""
    torch.manual_seed(60 + act)
    M, N, K = 1100, 512, 384
    fmt_a = no.E5M2 if act in (3, 5) else no.E4M3
    a8, dqa = no.quantize_fp8(torch.randn(M, K, device="cuda").to(torch.bfloat16), fmt_a)
    b8, dqb = no.quantize_fp8(torch.randn(N, K, device="cuda").to(torch.bfloat16) * 0.1, no.E4M3)
    z = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    bias = torch.randn(N, device="cuda") if act in (0, 4) else None
    kw = dict(fmt_a=fmt_a, bias=bias, act=act, addend=z if act != 4 else None)
    aux_r = torch.empty(M, N, dtype=torch.bfloat16, device="cuda") if act == 4 else None
    aux_1 = torch.empty_like(aux_r) if act == 4 else None
    ref = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    no.gemm_f8(a8, b8, ref, dqa, dqb, variant=1, aux=aux_1, **kw)
    out = torch.full((M, N), float("nan"), device="cuda").to(torch.bfloat16)
    no.gemm_f8(a8, b8, out, dqa, dqb, variant=12, aux=aux_r, **kw)
    torch.cuda.synchronize()
    assert nrmerr(out, ref) < 1e-2, nrmerr(out, ref)
    if act == 4:
        assert nrmerr(aux_r, aux_1) < 1e-2
    _, _, meta0 = no.quantize_fp8_delayed(torch.randn(M, N, device="cuda").to(torch.bfloat16), None, qfmt)
    q_ref, dq_ref, meta_ref = no.quantize_fp8_delayed(out, meta0.clone(), qfmt)
    codes = torch.empty(M, N, dtype=torch.uint8, device="cuda")
    meta = meta0.clone()
    out2 = torch.full_like(out, float("nan"))
    csum = torch.empty(N, dtype=torch.float32, device="cuda") if cs else None
    dq = no.gemm_f8(a8, b8, out2, dqa, dqb, variant=12, aux=torch.empty_like(out) if act == 4 else None,
                    q8=(codes, meta, qfmt, False), colsum_out=csum, **kw)
    torch.cuda.synchronize()
    assert torch.equal(out2, out)
    assert torch.equal(codes, q_ref), (codes != q_ref).sum().item()
    assert torch.equal(dq, dq_ref) and torch.equal(meta, meta_ref)
    if cs:
        assert nrmerr(csum, out.float().sum(0)) < 1e-3, nrmerr(csum, out.float().sum(0))


@pytest.mark.parametrize("act,qfmt,cs,K", [(None, 0, False, 384), (None, 1, False, 256), (4, 0, False, 384),
                                           (5, 1, True, 256), (0, 0, False, 256)])
def test_ring_persistent_matches_one_tile(act, qfmt, cs, K):
    """The persistent ring walk (fp8 variants 14 / 15: one workgroup per CU walks the tiles, the
    next tile's first K-tile prefetched under the current tile's epilogue) writes exactly the
    bytes of the one-tile launch (12 / 13): the plain GEMM (with / without bias, e4m3 / e5m2 A),
    and with the fused epilogues the bf16 output, gelu' side output, fp8 codes, dequant factor,
    amax history and column sums. 260 tiles (more than one per workgroup), a partial last tile
    row, an odd and an even K-tile count."""
    torch.manual_seed(80 + K)
    M, N = 16500, 1024
    fmt_a = no.E5M2 if (act in (3, 5) or (act is None and qfmt == 1)) else no.E4M3
    a8, dqa = no.quantize_fp8(torch.randn(M, K, device="cuda").to(torch.bfloat16), fmt_a)
    b8, dqb = no.quantize_fp8(torch.randn(N, K, device="cuda").to(torch.bfloat16) * 0.1, no.E4M3)
    if act is None:
        bias = torch.randn(N, device="cuda") if qfmt == 0 else None
        outs = {}
        for v in (12, 13, 14, 15):
            o = torch.full((M, N), float("nan"), device="cuda").to(torch.bfloat16)
            no.gemm_f8(a8, b8, o, dqa, dqb, fmt_a=fmt_a, bias=bias, variant=v)
            outs[v] = o
        torch.cuda.synchronize()
        assert torch.equal(outs[14], outs[12]) and torch.equal(outs[15], outs[13])
        assert torch.isfinite(outs[12].float()).all()
        return
    z = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    bias = torch.randn(N, device="cuda") if act in (0, 4) else None
    kw = dict(fmt_a=fmt_a, bias=bias, act=act, addend=z if act != 4 else None)
    _, _, meta0 = no.quantize_fp8_delayed(torch.randn(M, N, device="cuda").to(torch.bfloat16), None, qfmt)
    res = {}
    for v in (12, 14):
        out = torch.full((M, N), float("nan"), device="cuda").to(torch.bfloat16)
        aux = torch.full_like(out, float("nan")) if act == 4 else None
        codes = torch.empty(M, N, dtype=torch.uint8, device="cuda")
        meta = meta0.clone()
        csum = torch.empty(N, dtype=torch.float32, device="cuda") if cs else None
        dq = no.gemm_f8(a8, b8, out, dqa, dqb, variant=v, aux=aux, q8=(codes, meta, qfmt, False), colsum_out=csum,
                        **kw)
        res[v] = [out, codes, dq, meta] + ([aux] if aux is not None else []) + ([csum] if cs else [])
    torch.cuda.synchronize()
    for x, y in zip(res[14], res[12]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("T", [197, 50, 256, 7])
def test_cls_attention_kernel_matches_fp32(T):
    """csrc/attention_cls.hip: token 0's attention output and the full dqkv against an fp32
    torch reference of the same op."""
    torch.manual_seed(70 + T)
    B, H = 5, 12
    qkv = (torch.randn(B, T, 3 * H * 64, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_(True)
    o = fused.cls_attention(qkv, H)
    do = torch.randn_like(o)
    o.backward(do)
    ref_in = qkv.detach().float().requires_grad_(True)
    q, k, v = ref_in.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    p = torch.softmax((q[:, :, :1] @ k.transpose(-1, -2)) / 8.0, dim=-1)
    ref = (p @ v).transpose(1, 2).reshape(B, 1, H * 64)
    ref.backward(do.float())
    torch.cuda.synchronize()
    assert o.shape == (B, 1, H * 64)
    assert nrmerr(o, ref) < 1e-2, nrmerr(o, ref)
    g, gr = qkv.grad.view(B, T, 3, H * 64), ref_in.grad.view(B, T, 3, H * 64)
    assert torch.count_nonzero(g[:, 1:, 0]) == 0  # no query gradient except token 0's
    for i, name in enumerate("qkv"):
        e = nrmerr(g[:, :, i], gr[:, :, i])
        assert e < 2e-2, (name, e)


@pytest.mark.parametrize("fp8", [False, True])
def test_vit_cls_prune_native_matches_full(fp8, monkeypatch):
    """The native ViT with the class-token-only last block: loss and every parameter gradient
    close to the same model computing all 197 rows of the last block.

    bf16: the two arms directly, tight. fp8: each arm first runs three warm-up backward passes
    (weights unchanged) so its delayed scaling state has settled -- a fresh state quantises the
    first step with placeholder scales -- and then BOTH arms are compared with the bf16 model of
    the same weights: the pruned arm's error must stay within the full arm's error (plus a
    small margin) for every parameter. Measured (r6a): both arms sit 0.11-0.14 from bf16 on the
    first block's gradients (e5m2 output gradients keep 2 mantissa bits) and the pruned arm is
    never worse than the full one; the two fp8 arms then differ from each other by about the
    same 0.10-0.15 (independent rounding draws: the last block's scales see the class rows
    only), so a direct arm-to-arm bound measures quantisation noise, not the pruning."""
    from pytorch_distributed_template_amd.models.vit import VisionTransformer
    torch.manual_seed(3)
    m = VisionTransformer(depth=2, fp8=fp8).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 224, 224, device="cuda")
    y = torch.randint(0, 1000, (8,), device="cuda")

    def run(model, warm):
        for _ in range(warm):
            model.zero_grad(set_to_none=True)
            fused.softmax_cross_entropy(model(x), y).backward()
        model.zero_grad(set_to_none=True)
        loss = fused.softmax_cross_entropy(model(x), y)
        loss.backward()
        torch.cuda.synchronize()
        return float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters()}

    res = {}
    for prune in ("0", "1"):
        monkeypatch.setenv("PDT_VIT_CLS_PRUNE", prune)
        for mod in m.modules():  # fresh fp8 scaling state for each arm
            for a in ("_pdt_fp8_meta", "_pdt_fp8_gmeta"):
                if hasattr(mod, a):
                    delattr(mod, a)
        res[prune] = run(m, 3 if fp8 else 0)
    assert abs(res["1"][0] - res["0"][0]) < 2e-2 * abs(res["0"][0]), (res["1"][0], res["0"][0])
    if not fp8:
        for n, g in res["0"][1].items():
            e = nrmerr(res["1"][1][n], g)
            assert e < 2e-2, (n, e)
        return
    monkeypatch.setenv("PDT_VIT_CLS_PRUNE", "0")
    mb = VisionTransformer(depth=2, fp8=False).cuda().to(memory_format=torch.channels_last)
    mb.load_state_dict(m.state_dict())
    ref = run(mb, 0)[1]
    last = f"blocks.{len(m.blocks) - 1}."
    errs = {n: (nrmerr(res["0"][1][n], g), nrmerr(res["1"][1][n], g), nrmerr(res["1"][1][n], res["0"][1][n]))
            for n, g in ref.items()}
    msg = {n: tuple(round(v, 4) for v in e) for n, e in errs.items()}
    for n, (e_full, e_prune, _) in errs.items():
        assert e_full < 0.3, (n, msg)  # the fp8 path itself (both arms run it before the last block)
        assert e_prune < 1.25 * e_full + 0.03, (n, msg)
    # and the pruned last block's own parameters, where the arms compute differently
    assert any(n.startswith(last) for n in errs)


@pytest.mark.parametrize("rows,cols,fmt", [(50432, 768, 1), (4001, 2304, 1), (1000, 3072, 0), (777, 8, 1),
                                           (201728, 2304, 1)])
def test_cast_fp8_delayed_colsum(rows, cols, fmt):
    """pdt_cast_fp8_delayed_cs (row-grouped blocks, csrc/fp8.hip): codes bit-identical to the plain
    delayed cast from the same scaling state, the same amax-history roll, and column sums of
    the bf16 input (the bias gradient) against fp32. 50 432 and 201 728 rows (the ViT bs1024 qkv
    gradient) launch fewer bands than pdt_cast_cs_bands (whole rounds of resident blocks)."""
    torch.manual_seed(rows + cols)
    lib = no._load()
    x = (torch.randn(rows, cols, device="cuda") * 3).to(torch.bfloat16)
    _, _, meta = no.quantize_fp8_delayed(x, None, fmt)
    meta_a, meta_b = meta.clone(), meta.clone()
    q_ref = torch.empty(rows, cols, dtype=torch.uint8, device="cuda")
    dq_ref = torch.empty(1, dtype=torch.float32, device="cuda")
    no._chk(lib.pdt_cast_fp8_delayed(no._p(x), 1, x.numel(), no._p(meta_a), fmt, no._p(q_ref), no._p(dq_ref),
                                     no._s()), "cast_fp8_delayed")
    nb = lib.pdt_cast_cs_bands(rows)
    cpart = torch.empty(nb * cols + lib.pdt_reduce_rows_work(nb, cols), dtype=torch.float32, device="cuda")
    q = torch.empty(rows, cols, dtype=torch.uint8, device="cuda")
    dq = torch.empty(1, dtype=torch.float32, device="cuda")
    db = torch.empty(cols, dtype=torch.float32, device="cuda")
    no._chk(lib.pdt_cast_fp8_delayed_cs(no._p(x), rows, cols, no._p(meta_b), fmt, no._p(q), no._p(dq), no._p(cpart),
                                        no._p(db), no._s()), "cast_fp8_delayed_cs")
    torch.cuda.synchronize()
    assert torch.equal(q, q_ref)
    assert torch.equal(dq, dq_ref)
    assert torch.equal(meta_a, meta_b)
    ref = x.float().sum(0)
    assert ((db - ref).norm() / ref.norm()).item() < 1e-5


def test_linear_wgrad_bias_without_param():
    """_linear_wgrad(..., with_bias=True) without a bias tensor: the bias-gradient buffer is
    allocated on the GPU (ops/native_ops.py _grad_buf). With device=None it landed on the host
    and the weight-gradient kernel wrote through a host pointer -- the illegal access that
    faulted round 5's r5z variant sweep."""
    torch.manual_seed(3)
    M, Nout, K = 1000, 256, 128
    dy = torch.randn(M, Nout, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.empty(Nout, K, device="cuda")
    dw, db = no._linear_wgrad(dy, x, w, with_bias=True)
    torch.cuda.synchronize()
    assert db.is_cuda and dw.is_cuda
    assert nrmerr(db, dy.float().sum(0)) < 1e-5
    assert nrmerr(dw, dy.float().t() @ x.float()) < 1e-3


def test_vit_ln_codes_only_output_bit_identical(monkeypatch):
    """fp8 ViT with the LayerNorm outputs written as e4m3 codes only (their consumers, qkv and
    fc1, read nothing else: ops/native_ops.py _ln_codes_only) against the same step with the bf16
    outputs written too: loss and every parameter gradient bit-identical from the same weights
    and fp8 scaling state, and the codes-only launches actually taken."""
    from pytorch_distributed_template_amd.models.vit import VisionTransformer
    torch.manual_seed(4)
    m = VisionTransformer(depth=2, fp8=True).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 224, 224, device="cuda")
    y = torch.randint(0, 1000, (8,), device="cuda")
    monkeypatch.setenv("PDT_LN_CODES_ONLY", "0")
    for _ in range(3):  # delayed-scaling histories exist from here on: the LayerNorms emit codes
        m.zero_grad(set_to_none=True)
        fused.softmax_cross_entropy(m(x), y).backward()
    names = ("_pdt_fp8_meta", "_pdt_fp8_gmeta")
    state = [(mod, a, getattr(mod, a).clone()) for mod in m.modules() for a in names if hasattr(mod, a)]
    assert state
    lib = no._load()
    seen = {"null_y": 0}
    for fn_name, y_arg in (("pdt_ln_fwd_f8", 3), ("pdt_ln_add_fwd", 5)):
        orig = getattr(lib, fn_name)

        def wrap(*a, orig=orig, y_arg=y_arg):
            seen["null_y"] += a[y_arg] is None
            return orig(*a)
        monkeypatch.setattr(lib, fn_name, wrap)
    res = {}
    for only in ("0", "1"):
        for mod, a, t in state:
            getattr(mod, a).copy_(t)
        monkeypatch.setenv("PDT_LN_CODES_ONLY", only)
        seen["null_y"] = 0
        m.zero_grad(set_to_none=True)
        loss = fused.softmax_cross_entropy(m(x), y)
        loss.backward()
        torch.cuda.synchronize()
        res[only] = (float(loss), {n: p.grad.clone() for n, p in m.named_parameters()}, seen["null_y"])
    assert res["0"][2] == 0 and res["1"][2] >= 4, (res["0"][2], res["1"][2])  # 2 LayerNorms per block
    assert res["1"][0] == res["0"][0]
    for n, g in res["0"][1].items():
        assert torch.equal(res["1"][1][n], g), n

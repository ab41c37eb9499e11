"""Persistent ring tiles of the implicit-GEMM kernel (csrc/conv_nt_kernel.h PERS, variant ids
after the halo kernels): one workgroup per CU walks several output tiles, so the shapes here
have well over 256 tiles of every tile size -- the tile loop, the LDS hand-over between tiles
and the per-tile epilogues (BN statistics partials, fused BN-backward partials) all run more
than once per workgroup. Each variant is checked against an fp32 matmul of the same bf16
operands, and against the non-persistent variant of the same tile bit for bit."""
import pytest
import torch

from pytorch_distributed_template_amd.ops import native_ops as no

pytestmark = pytest.mark.gpu

PERS_BASE = {0: 34, 1: 35, 2: 36}  # persistent id - PERS0 -> its tile's one-shot variant
BNB_ONLY = {2}  # the persistent 256x256 ring carries the BN-backward epilogue only


def _pers_ids(lib):
    nvar = lib.pdt_conv_nt_num_variants()
    kinds = [lib.pdt_conv_nt_variant_kind(v) for v in range(nvar)]
    halo_end = max(v for v in range(nvar) if kinds[v] == 2) + 1
    return list(range(halo_end, nvar))


def _geom(M, N, K):
    return dict(Hs=1, Ws=1, Cs=K, Nimg=M, Hm=1, Wm=1, Ncol=N, K=K, ldb=K, sh=1, sw=1, oh0=0, ow0=0, dh=1, dw=1,
                nth=1, ntw=1, Ho=1, Wo=1, osh=1, osw=1, oph=0, opw=0, ldo=N)


def nrmerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,N,K", [(256 * 301, 512, 384), (256 * 150 + 77, 768, 192)])
def test_persistent_ring_tiles_forward_and_stats(M, N, K):
    lib = no._load()
    pers = _pers_ids(lib)
    assert len(pers) == len(PERS_BASE)
    torch.manual_seed(5)
    dev = "cuda"
    a_ = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b_ = torch.randn(N, K, device=dev).to(torch.bfloat16)
    ref = a_.float() @ b_.float().t()
    g = _geom(M, N, K)
    for i, v in enumerate(pers):
        rows = lib.pdt_conv_nt_stat_rows(M, N, K, v)
        assert rows == lib.pdt_conv_nt_stat_rows(M, N, K, PERS_BASE[i])
        part = torch.full((2 * rows * N,), float("nan"), device=dev)
        out = torch.full((M, N), float("nan"), device=dev).to(torch.bfloat16)
        rc = lib.pdt_conv_nt(*no._nt_args(a_, b_, out, part, None, g, 0, v))
        if i in BNB_ONLY:
            assert rc == no.NOT_APPLICABLE, (v, rc)
            continue
        assert rc == 0, (v, rc)
        torch.cuda.synchronize()
        assert nrmerr(out, ref) < 1e-2, v
        ps = part.view(2, rows, N).sum(1)
        assert nrmerr(ps[0], ref.sum(0)) < 1e-3, v
        assert nrmerr(ps[1], (ref * ref).sum(0)) < 1e-3, v
        # the same tile computed one tile per workgroup: identical bits
        out1 = torch.empty_like(out)
        part1 = torch.empty_like(part)
        assert lib.pdt_conv_nt(*no._nt_args(a_, b_, out1, part1, None, g, 0, PERS_BASE[i])) == 0
        assert torch.equal(out, out1), v
        assert torch.equal(part, part1), v


@pytest.mark.parametrize("block_input", [False, True])
def test_persistent_ring_tiles_bn_backward_epilogue(block_input):
    """The fused BN-backward partials (pdt_conv_nt_bnb) from the persistent tiles: every tile
    writes its own partial row, in the two configurations the ring tiles compile -- a block's
    inner unit (ReLU gate recomputed from y) and a block input (ReLU-masked addend, the
    unit's ReLU bit mask)."""
    lib = no._load()
    torch.manual_seed(6)
    dev = "cuda"
    M, N, K = 256 * 280, 256, 256
    dy = torch.randn(M, K, device=dev).to(torch.bfloat16)
    wt = torch.randn(N, K, device=dev).to(torch.bfloat16)
    y = torch.randn(M, N, device=dev).to(torch.bfloat16)
    mean = torch.randn(N, device=dev) * 0.1
    scale = torch.rand(N, device=dev) + 0.5
    shift = torch.randn(N, device=dev) * 0.1
    add = torch.randn(M, N, device=dev).to(torch.bfloat16) if block_input else None
    amask = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device=dev) if block_input else None
    bmask = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device=dev) if block_input else None

    def bits(m):
        return ((m.view(-1, 1).int() >> torch.arange(8, device=dev)) & 1).view(M, N).float()

    ref = dy.float() @ wt.float().t()
    if block_input:
        ref = ref + add.float() * bits(amask)
        gate = bits(bmask)
    else:
        gate = ((y.float() * scale + shift) > 0).float()
    def run(v):
        R = lib.pdt_conv_nt_bnb_rows(M, N, K, v)
        part = torch.full((2 * R * N,), float("nan"), device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        rc = lib.pdt_conv_nt_bnb(no._p(dy), no._p(wt), no._p(out), no._p(add), no._p(amask),
                                 1, 1, K, M, 1, 1, N, K, K, 1, 1, 0, 0, 1, 1, 1, 1,
                                 1, 1, 1, 1, 0, 0, N, v, no._p(y), no._p(mean), no._p(scale), no._p(shift),
                                 no._p(bmask), no._p(part), 1, 0, R, no._s())
        assert rc == 0, (v, rc)
        torch.cuda.synchronize()
        return out, part, R

    for i, v in enumerate(_pers_ids(lib)):
        out, part, R = run(v)
        assert nrmerr(out, ref) < 1e-2, v
        gg = out.float() * gate
        ps = part.view(2, R, N).sum(1)
        assert nrmerr(ps[0], gg.sum(0)) < 1e-3, v
        assert nrmerr(ps[1], (gg * (y.float() - mean)).sum(0)) < 1e-3, v
        out1, part1, _ = run(PERS_BASE[i])  # the same tile one per workgroup: identical bits
        assert torch.equal(out, out1) and torch.equal(part, part1), v

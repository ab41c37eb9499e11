"""A/B of the fp8 dense ring launched one tile per workgroup (gemm_f8 variants 12 / 13) against
the persistent walk (14 / 15: the next tile's first K-tile loads under the current tile's
epilogue) on the ViT-B/16 bs1024 GEMM shapes: the plain GEMMs, fc1's fused epilogue (GELU +
GELU' + e4m3 codes) and fc2's data-gradient epilogue (x gelu' + e5m2 codes + column sums).
Interleaved rounds, median per variant; outputs are compared bit for bit with variant 12's.

    python scripts/ring_pers_ab.py [M]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 201728
    torch.manual_seed(0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timeit(fn, reps=5):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    def ab(name, flops, make, variants):
        runs = {v: make(v) for v in variants}
        outs = {}
        for v, (fn, res) in runs.items():
            fn()
            torch.cuda.synchronize()
            outs[v] = [t.clone() for t in res()]
        t = {v: [] for v in variants}
        for _ in range(5):
            for v, (fn, _) in runs.items():
                t[v].append(timeit(fn))
        line = f"{name}:"
        for v in variants:
            med = statistics.median(t[v])
            line += f"  v{v} {med * 1e3:7.1f} us ({flops / med / 1e9:5.0f} TF)"
        ref = outs[variants[0]]
        for v in variants[1:]:
            same = all(torch.equal(a, b) for a, b in zip(outs[v], ref))
            line += f"  v{v}{'==' if same else '!='}v{variants[0]}"
        print(line, flush=True)

    for N, K, fmt in ((2304, 768, no.E4M3), (768, 768, no.E4M3), (3072, 768, no.E4M3), (768, 3072, no.E4M3),
                      (768, 2304, no.E5M2), (3072, 768, no.E5M2), (768, 768, no.E5M2)):
        a8, dqa = no.quantize_fp8(torch.randn(M, K, device="cuda").to(torch.bfloat16), fmt)
        b8, dqb = no.quantize_fp8((torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16), no.E4M3)
        bias = torch.randn(N, device="cuda") if fmt == no.E4M3 else None
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")

        def plain(v, a8=a8, b8=b8, dqa=dqa, dqb=dqb, fmt=fmt, bias=bias, out=out):
            return (lambda: no.gemm_f8(a8, b8, out, dqa, dqb, fmt_a=fmt, bias=bias, variant=v)), (lambda: [out])

        ab(f"plain {'e4m3' if fmt == no.E4M3 else 'e5m2'} M={M} N={N} K={K}", 2.0 * M * N * K, plain, [12, 13, 14, 15])
        del a8, b8, out
    # fc1 forward: x[M, 768] W1[3072, 768]^T + b1 -> gelu' (aux), e4m3 codes of gelu (q8, only)
    x8, dqx = no.quantize_fp8(torch.randn(M, 768, device="cuda").to(torch.bfloat16), no.E4M3)
    w8, dqw = no.quantize_fp8((torch.randn(3072, 768, device="cuda") * 0.05).to(torch.bfloat16), no.E4M3)
    b1 = torch.randn(3072, device="cuda") * 0.1
    _, _, meta = no.quantize_fp8_delayed(torch.randn(M, 3072, device="cuda").to(torch.bfloat16), None, no.E4M3)
    a = torch.empty(M, 3072, dtype=torch.bfloat16, device="cuda")
    z = torch.empty_like(a)
    aq = torch.empty(M, 3072, dtype=torch.uint8, device="cuda")
    metas = {}

    def fc1(v):
        m = metas.setdefault(("fc1", v), meta.clone())

        def fn():
            m.copy_(meta)
            no.gemm_f8(x8, w8, a, dqx, dqw, bias=b1, act=no.ACT_GELU_DUAL, aux=z, q8=(aq, m, no.E4M3, True),
                       variant=v)
        return fn, (lambda: [z, aq, m])

    ab(f"fc1 epilogue M={M} N=3072 K=768", 2.0 * M * 3072 * 768, fc1, [12, 14])
    del x8, a, aq
    # fc2 data gradient: g[M, 768] e5m2 x W2^T[3072, 768] -> x gelu'(z), e5m2 codes, column sums
    g8, dqg = no.quantize_fp8(torch.randn(M, 768, device="cuda").to(torch.bfloat16), no.E5M2)
    dz = torch.empty(M, 3072, dtype=torch.bfloat16, device="cuda")
    dzq = torch.empty(M, 3072, dtype=torch.uint8, device="cuda")
    _, _, gmeta = no.quantize_fp8_delayed(torch.randn(M, 3072, device="cuda").to(torch.bfloat16) * 1e-3, None,
                                          no.E5M2)
    db = torch.empty(3072, device="cuda")

    def fc2(v):
        m = metas.setdefault(("fc2", v), gmeta.clone())

        def fn():
            m.copy_(gmeta)
            no.gemm_f8(g8, w8, dz, dqg, dqw, fmt_a=no.E5M2, act=no.ACT_MUL, addend=z, q8=(dzq, m, no.E5M2, True),
                       colsum_out=db, variant=v)
        return fn, (lambda: [dzq, m, db])

    ab(f"fc2 dgrad epilogue M={M} N=3072 K=768", 2.0 * M * 3072 * 768, fc2, [12, 14])


if __name__ == "__main__":
    main()

"""GEMM throughput on the ViT-B/16 (batch 256) linear shapes: native bf16
conv_nt GEMM (every tile variant), native fp8 GEMM (every variant), and the
library paths torch.matmul (hipBLASLt) / torch._scaled_mm for reference.

    python scripts/bench_gemm.py [--iters 10] [--shapes vit|resnet]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

SHAPES = [  # M, N, K  (tokens x out x in)
    (50432, 2304, 768),   # qkv
    (50432, 768, 768),    # proj
    (50432, 3072, 768),   # fc1
    (50432, 768, 3072),   # fc2
    (50432, 768, 2304),   # qkv dgrad
    (50432, 3072, 768),   # fc2 dgrad (K=768 -> N=3072)
]
RESNET_SHAPES = [  # 1x1 convs of ResNet-50 at 2048 images as plain GEMMs (pixels x Cout x Cin) + the square reference
    (401408, 256, 1024), (401408, 1024, 256), (100352, 512, 2048), (100352, 2048, 512),
    (1605632, 128, 512), (1605632, 512, 128), (8192, 8192, 8192),
]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="vit", choices=["vit", "resnet"])
    ap.add_argument("--variants", default="", help="also print these bf16 variant ids' own times (e.g. 36,37,45,46)")
    a = ap.parse_args()
    lib = no._load()
    for M, N, K in (SHAPES if a.shapes == "vit" else RESNET_SHAPES):
        fl = 2.0 * M * N * K
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        geo = dict(Hs=1, Ws=1, Cs=K, Nimg=M, Hm=1, Wm=1, Ncol=N, K=K, ldb=K, sh=1, sw=1, oh0=0, ow0=0, dh=1, dw=1,
                   nth=1, ntw=1, Ho=1, Wo=1, osh=1, osw=1, oph=0, opw=0, ldo=N)
        best = (1e9, -1)
        per_v = {}
        for v in range(lib.pdt_conv_nt_num_variants()):
            if lib.pdt_conv_nt(*no._nt_args(x, w, y, None, None, geo, 0, v)) == no.NOT_APPLICABLE:
                continue
            t = timeit(lambda: no.conv_nt(x, w, y, variant=v, **geo), a.iters)
            per_v[v] = t
            best = min(best, (t, v))
        if a.variants:
            print(f"M={M} N={N} K={K}: " + "  ".join(
                f"v{v} {per_v[int(v)] * 1e3:.1f} us" for v in a.variants.split(",") if int(v) in per_v), flush=True)
        t_lib = timeit(lambda: torch.matmul(x, w.t()), a.iters)
        xq, dqx = no.quantize_fp8(x)
        wq, dqw = no.quantize_fp8(w)
        best8 = (1e9, -1)
        for v in range(lib.pdt_gemm_f8_num_variants()):
            try:
                t = timeit(lambda: no.gemm_f8(xq, wq, y, dqx, dqw, variant=v), a.iters)
            except no.NotApplicable:  # (the dense ring: N % 256 == 0)
                continue
            best8 = min(best8, (t, v))
        # the dense bf16 ring (csrc/gemm_ring.hip, groupings GM 4 / 8)
        ring = (1e9, -1)
        for sub in range(2):
            if lib.pdt_gemm_ring(no._p(x), no._p(w), no._p(y), None, None, None, M, N, K, K, K, N, 0, sub,
                                 no._s()) != 0:
                continue
            t = timeit(lambda: lib.pdt_gemm_ring(no._p(x), no._p(w), no._p(y), None, None, None, M, N, K, K, K, N, 0,
                                                 sub, no._s()), a.iters)
            ring = min(ring, (t, sub))
        t_q = timeit(lambda: no.quantize_fp8(x), a.iters)
        line = (f"M={M} N={N} K={K}: native bf16 {best[0] * 1e3:7.1f} us ({fl / best[0] / 1e9:6.0f} TF, v{best[1]})"
                f" | ring bf16 " + (f"{ring[0] * 1e3:7.1f} us ({fl / ring[0] / 1e9:6.0f} TF, gm{4 * (1 + ring[1])})"
                                      if ring[1] >= 0 else "n/a") +
                f" | hipBLASLt bf16 {t_lib * 1e3:7.1f} us ({fl / t_lib / 1e9:6.0f} TF)"
                f" | native fp8 {best8[0] * 1e3:7.1f} us ({fl / best8[0] / 1e9:6.0f} TF, v{best8[1]})"
                f" | quantize x {t_q * 1e3:6.1f} us")
        try:
            xs = xq.view(torch.float8_e4m3fn)
            ws = wq.view(torch.float8_e4m3fn)
            one = torch.ones((), device="cuda")
            t_s = timeit(lambda: torch._scaled_mm(xs, ws.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16),
                         a.iters)
            line += f" | _scaled_mm fp8 {t_s * 1e3:7.1f} us ({fl / t_s / 1e9:6.0f} TF)"
        except Exception as e:  # noqa: BLE001
            line += f" | _scaled_mm n/a ({type(e).__name__})"
        print(line, flush=True)


if __name__ == "__main__":
    main()

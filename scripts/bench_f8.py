"""fp8 GEMM variants on the ViT-B/16 batch-1024 linear shapes (M = 1024 * 197 tokens):
every forward / data-gradient tile of pdt_gemm_f8 and every weight-gradient tile of
pdt_linear_wgrad_f8, each checked against variant 10 (the 8-wave 256x256 ring), plus
torch._scaled_mm (hipBLASLt) on the same codes for reference.

    python scripts/bench_f8.py [--iters 10] [--fwd 8,10,11] [--wgrad 10,12,21,22,23,24]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

M = 1024 * 197
FWD = [(2304, 768), (768, 768), (3072, 768), (768, 3072), (768, 2304)]  # (N, K): qkv, proj, fc1, fc2, qkv dgrad
WG = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]                 # (Nout, K)


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


def nrmerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--fwd", default="8,9,10,11")
    ap.add_argument("--wgrad", default="10,12,19,20,21,22,23,24")
    ap.add_argument("--bias", action="store_true", help="weight gradients with the bias gradient (bf16 dY column sums)")
    a = ap.parse_args()
    torch.manual_seed(0)
    # ("+" also separates ids: scripts/gpu_job.sh turns commas into spaces)
    fv = [int(v) for v in a.fwd.replace("+", ",").split(",") if v]
    wv = [int(v) for v in a.wgrad.replace("+", ",").split(",") if v]
    for N, K in FWD:
        fl = 2.0 * M * N * K
        xq, dqx = no.quantize_fp8(torch.randn(M, K, device="cuda").to(torch.bfloat16))
        wq, dqw = no.quantize_fp8(torch.randn(N, K, device="cuda").to(torch.bfloat16))
        ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        no.gemm_f8(xq, wq, ref, dqx, dqw, variant=10)
        parts = []
        for v in fv:
            y = torch.empty_like(ref)
            try:
                t = timeit(lambda: no.gemm_f8(xq, wq, y, dqx, dqw, variant=v), a.iters)
            except no.NotApplicable:
                continue
            parts.append(f"v{v} {t * 1e3:6.1f} us {fl / t / 1e9:5.0f} TF err {nrmerr(y, ref):.1e}")
        one = torch.ones((), device="cuda")
        xs, ws = xq.view(torch.float8_e4m3fn), wq.view(torch.float8_e4m3fn)
        t_s = timeit(lambda: torch._scaled_mm(xs, ws.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16),
                     a.iters)
        parts.append(f"_scaled_mm {t_s * 1e3:6.1f} us {fl / t_s / 1e9:5.0f} TF")
        print(f"fwd M={M} N={N} K={K}: " + " | ".join(parts), flush=True)
        del xq, wq, ref
    for Nout, K in WG:
        fl = 2.0 * M * Nout * K
        dyq, dqd = no.quantize_fp8(torch.randn(M, Nout, device="cuda").to(torch.bfloat16), no.E5M2)
        xq, dqx = no.quantize_fp8(torch.randn(M, K, device="cuda").to(torch.bfloat16))
        dy16 = torch.randn(M, Nout, device="cuda").to(torch.bfloat16) if a.bias else None
        ref, _ = no.linear_wgrad_f8(dyq, xq, dqd, dqx, variant=10)
        ref = ref.clone()
        parts = []
        for v in wv:
            out = {}

            def run():
                out["dw"], _ = no.linear_wgrad_f8(dyq, xq, dqd, dqx, dy16=dy16, with_bias=a.bias, variant=v)

            t = timeit(run, a.iters)
            parts.append(f"v{v} {t * 1e3:6.1f} us {fl / t / 1e9:5.0f} TF err {nrmerr(out['dw'], ref):.1e}")
        print(f"wgrad M={M} Nout={Nout} K={K}: " + " | ".join(parts), flush=True)
        del dyq, xq


if __name__ == "__main__":
    main()

"""Which fp8 layouts / epilogues torch._scaled_mm (hipBLASLt) takes on this box, and how fast,
on the ViT-B/16 batch-1024 GEMMs, next to the tuned native kernel of the same call:

  dgrad  e5m2 dY [M][N] x e4m3 W [N][K]  (A row-major, B = W as stored: column-major [N][K]^T)
  fwd    e4m3 X x e4m3 W + bf16 bias
  wgrad  dW[Nout][K] = dY^T X: A = dY^T (column-major view), B = X (row-major)

    python scripts/probe_scaled_mm.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

M = 1024 * 197
E4, E5 = torch.float8_e4m3fn, torch.float8_e5m2


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def nrmerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def q(x, fmt):
    return no.quantize_fp8(x.to(torch.bfloat16), fmt)


def try_(label, fn, ref=None, fl=None):
    try:
        out = fn()
        t = timeit(fn)
        err = f" err {nrmerr(out, ref):.1e}" if ref is not None else ""
        tf = f" {fl / t / 1e6:5.0f} TF" if fl else ""
        print(f"  {label:44s} {t:8.1f} us{tf}{err}", flush=True)
        return t
    except Exception as e:  # noqa: BLE001
        print(f"  {label:44s} n/a: {type(e).__name__}: {str(e).splitlines()[0][:150]}", flush=True)
        return None


def main():
    torch.manual_seed(0)
    dev = "cuda"
    one = torch.ones((), device=dev)
    print("dgrad (e5m2 dY x e4m3 W):")
    for N, K in [(768, 3072), (768, 768), (768, 2304), (3072, 768)]:
        # out[M][K] = dY[M][N] @ W[N][K]; native pdt_gemm_f8 takes b = W^T as [K][N] (wqt)
        dyq, dqd = q(torch.randn(M, N, device=dev), no.E5M2)
        wtq, dqw = q(torch.randn(K, N, device=dev), no.E4M3)  # [K][N] = the native B
        out = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        print(f" M={M} N(out)={K} K(red)={N}")
        tn = try_("native (tuned)", lambda: no.gemm_f8(dyq, wtq, out, dqd, dqw, fmt_a=no.E5M2), fl=fl)
        ref = out.clone()
        try_("_scaled_mm e5m2 x e4m3", lambda: torch._scaled_mm(dyq.view(E5), wtq.view(E4).t(), scale_a=dqd,
                                                                 scale_b=dqw, out_dtype=torch.bfloat16), ref, fl)
        _ = tn
        del dyq, wtq, out
    print("fwd + bias (e4m3 x e4m3):")
    for N, K in [(2304, 768), (768, 3072), (768, 768)]:
        xq, dqx = q(torch.randn(M, K, device=dev), no.E4M3)
        wq, dqw = q(torch.randn(N, K, device=dev), no.E4M3)
        bias = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        print(f" M={M} N={N} K={K}")
        try_("native (tuned) + fp32 bias", lambda: no.gemm_f8(xq, wq, out, dqx, dqw, bias=bias), fl=fl)
        ref = out.clone()
        bb = bias.to(torch.bfloat16)
        try_("_scaled_mm + bf16 bias", lambda: torch._scaled_mm(xq.view(E4), wq.view(E4).t(), scale_a=dqx,
                                                                 scale_b=dqw, bias=bb, out_dtype=torch.bfloat16),
             ref, fl)
        try_("_scaled_mm out= (no bias)", lambda: torch._scaled_mm(xq.view(E4), wq.view(E4).t(), scale_a=dqx,
                                                                    scale_b=dqw, out_dtype=torch.bfloat16,
                                                                    out=out), None, fl)
        del xq, wq, out
    print("wgrad (dW = dY^T X):")
    for Nout, K in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
        dyq, dqd = q(torch.randn(M, Nout, device=dev), no.E5M2)
        xq, dqx = q(torch.randn(M, K, device=dev), no.E4M3)
        fl = 2.0 * M * Nout * K
        print(f" M(red)={M} Nout={Nout} K={K}")
        res = {}

        def nat():
            res["dw"], _ = no.linear_wgrad_f8(dyq, xq, dqd, dqx)
            return res["dw"]

        try_("native (tuned) fp32 dW", nat, fl=fl)
        ref = res["dw"].clone()
        try_("_scaled_mm A=dY^T(col) B=X(row) -> fp32", lambda: torch._scaled_mm(
            dyq.view(E5).t(), xq.view(E4), scale_a=dqd, scale_b=dqx, out_dtype=torch.float32), ref, fl)
        try_("_scaled_mm A=dY^T(col) B=X(row) -> bf16", lambda: torch._scaled_mm(
            dyq.view(E5).t(), xq.view(E4), scale_a=dqd, scale_b=dqx, out_dtype=torch.bfloat16), ref, fl)
        dyt = dyq.t().contiguous()
        xt = xq.t().contiguous()
        try_("transpose copies of both codes", lambda: (dyq.t().contiguous(), xq.t().contiguous()))
        try_("_scaled_mm dY^T(row) x X^T(col) -> fp32", lambda: torch._scaled_mm(
            dyt.view(E5), xt.view(E4).t(), scale_a=dqd, scale_b=dqx, out_dtype=torch.float32), ref, fl)
        del dyq, xq, dyt, xt


if __name__ == "__main__":
    main()

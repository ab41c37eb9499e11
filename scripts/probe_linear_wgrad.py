"""ViT-B/16 linear weight-gradient shapes (M = 256 * 197 tokens): native split-K
wgrad vs the library GEMM (hipBLASLt through torch.mm) with fp32 and bf16
outputs, and the library data gradient for scale. Prints microseconds and TF/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    M = 256 * 197
    for nout, k in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        dy = torch.randn(M, nout, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, k, device="cuda").to(torch.bfloat16)
        w = torch.randn(nout, k, device="cuda")
        flop = 2.0 * M * nout * k
        tn = timeit(lambda: no._linear_wgrad_native(dy, x, w))
        tl32 = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        tl16 = timeit(lambda: torch.mm(dy.t(), x))
        tlt = timeit(lambda: torch.mm(x.t(), dy))
        td = timeit(lambda: torch.mm(dy, w.to(torch.bfloat16)))
        ref = torch.mm(dy.float().t(), x.float())
        e32 = ((torch.mm(dy.t(), x, out_dtype=torch.float32) - ref).norm() / ref.norm()).item()
        en = ((no._linear_wgrad_native(dy, x, w) - ref).norm() / ref.norm()).item()
        print(f"{nout}x{k}: native {tn:7.1f} us ({flop / tn / 1e6:6.1f} TF/s, err {en:.2e}) | "
              f"lib fp32-out {tl32:7.1f} ({flop / tl32 / 1e6:6.1f}, err {e32:.2e}) | lib bf16-out {tl16:7.1f} "
              f"({flop / tl16 / 1e6:6.1f}) | lib x^T dy bf16 {tlt:7.1f} | lib dgrad {td:7.1f} ({flop / td / 1e6:6.1f})",
              flush=True)


if __name__ == "__main__":
    main()

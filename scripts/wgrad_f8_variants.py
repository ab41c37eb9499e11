"""Time every fp8 weight-gradient variant (csrc/wgrad_f8.hip) on the ViT-B/16 bs256 linear
shapes (M tokens, default 50432 = bs256; 201728 = bs1024) against the bf16 weight
gradient's best variant.

    python scripts/wgrad_f8_variants.py [M]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def timed(fn, n=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    lib = no._load()
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 50432
    tot8 = tot16 = 0.0
    for Mo, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        dy = torch.randn(M, Mo, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        dyq, dqdy = no.quantize_fp8(dy, no.E5M2)
        xq, dqx = no.quantize_fp8(x, no.E4M3)
        t8 = {v: timed(lambda: no.linear_wgrad_f8(dyq, xq, dqdy, dqx, dy16=dy, with_bias=True, variant=v))
              for v in range(lib.pdt_wgrad_f8_num_variants())}
        t16 = timed(lambda: no._linear_wgrad(dy, x, torch.empty(Mo, K, device="cuda"), with_bias=True))
        fl = 2.0 * M * Mo * K
        b = min(t8, key=t8.get)
        tot8 += t8[b]
        tot16 += t16
        print(f"{Mo}x{K}: bf16 {t16 * 1e3:7.1f} us ({fl / t16 / 1e9:5.0f} TF) | fp8 best v{b} {t8[b] * 1e3:7.1f} us "
              f"({fl / t8[b] / 1e9:5.0f} TF)  all: " + " ".join(f"{v}:{t * 1e3:.0f}" for v, t in t8.items()), flush=True)
    print(f"per block: bf16 {tot16:.3f} ms, fp8 {tot8:.3f} ms")


if __name__ == "__main__":
    main()

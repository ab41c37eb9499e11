"""Times the halo stem kernels (csrc/stem.hip) at the bench geometry against each other:
forward, and the weight-gradient variants (pdt_stem_wgrad_v 0 / 1, slab reduce included).

    python scripts/stem_bench.py [--batch 2048] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


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
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    lib = no._load()
    dev = "cuda"
    N, H, W = a.batch, 224, 224
    x4 = torch.randn(N, H, W, 4, device=dev).to(torch.bfloat16)
    w = torch.randn(64, 3, 7, 7, device=dev) * 0.1
    wb = no._s2d_weight(w)
    y = torch.empty(N, H // 2, W // 2, 64, device=dev, dtype=torch.bfloat16)
    R = lib.pdt_stem_fwd_rows(N, H, W, 64)
    part = torch.empty(2 * R * 64, device=dev)
    t = timeit(lambda: lib.pdt_stem_fwd(no._p(x4), no._p(wb), no._p(y), no._p(part), N, H, W, 64, no._s()), a.iters)
    print(f"stem forward (halo)          {t * 1e3:8.1f} us", flush=True)
    dA = torch.randn_like(y, dtype=torch.float32).to(torch.bfloat16)
    coef = torch.rand(5, 64, device=dev).contiguous()
    dw = torch.empty(64, 256, device=dev)
    for v in (0, 1):
        splits = lib.pdt_stem_wgrad_splits_v(N, H, W, 64, v)
        ws = torch.empty(lib.pdt_wgrad_workspace(splits, 64, 256), device=dev)

        def run():
            lib.pdt_stem_wgrad_v(no._p(x4), no._p(dA), no._p(y), no._p(coef), no._p(ws), N, H, W, 64, v, no._s())
            lib.pdt_wgrad_reduce(no._p(ws), no._p(dw), None, None, splits, 64, 256, 1.0, 0, no._s())
        t = timeit(run, a.iters)
        print(f"stem weight gradient v{v}      {t * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()

"""Time every conv_nt tile variant (and the halo kernels) on the ResNet-50 3x3 stride-1
forward shapes (with BN statistics) at batch 2048 (argv[1]: another batch); prints all
variants sorted with achieved TFLOP/s, so the tuner's pick can be compared with the
256x256 ring tiles (ids 36, 37)."""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

SHAPES = [(64, 56), (128, 28), (256, 14), (512, 7)]  # C (in = out), H


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    lib = no._load()
    nvar = lib.pdt_conv_nt_num_variants()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for C, H in SHAPES:
        conv = nn.Conv2d(C, C, 3, 1, 1, bias=False).cuda().to(memory_format=torch.channels_last)
        x = (torch.rand(n, C, H, H, device="cuda") * 2 - 1).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        g = no._fwd_geom(n, H, H, C, conv)
        a = no._fwd_nt_geom(n, H, H, C, C, g)
        wb = no.bf16_weight(conv.weight)
        M = n * H * H
        K = a["K"]
        flop = 2.0 * M * C * K
        y = torch.empty((n, C, H, H), dtype=torch.bfloat16, device="cuda", memory_format=torch.channels_last)
        res = []
        for v in range(nvar):
            R = max(lib.pdt_conv_nt_stat_rows(M, C, K, v), 1)
            st = torch.empty(2 * R * C, device="cuda")
            args = no._nt_args(x, wb, y, st, None, a, 0, v)
            rc = lib.pdt_conv_nt(*args)
            if rc != 0:
                continue
            best = float("inf")
            for _ in range(3):
                ev0.record()
                for _ in range(5):
                    lib.pdt_conv_nt(*args)
                ev1.record()
                ev1.synchronize()
                best = min(best, ev0.elapsed_time(ev1) / 5 * 1e3)
            res.append((best, v))
        res.sort()
        line = " ".join(f"v{v}:{t:.0f}us/{flop / t / 1e6:.0f}TF" for t, v in res)
        print(f"n={n} C={C} H={H} K={K}: {line}", flush=True)


def square(n=8192):
    """The plain-GEMM reference point: M = N = K = n (a 1x1 conv over n 1x1 images)."""
    lib = no._load()
    nvar = lib.pdt_conv_nt_num_variants()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    conv = nn.Conv2d(n, n, 1, 1, 0, bias=False).cuda().to(memory_format=torch.channels_last)
    x = (torch.rand(n, n, 1, 1, device="cuda") * 2 - 1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = no._fwd_geom(n, 1, 1, n, conv)
    a = no._fwd_nt_geom(n, 1, 1, n, n, g)
    wb = no.bf16_weight(conv.weight)
    y = torch.empty((n, n, 1, 1), dtype=torch.bfloat16, device="cuda", memory_format=torch.channels_last)
    res = []
    for v in (0, 5, 20, 25, 30, 31, 34, 35, 36, 37):
        args = no._nt_args(x, wb, y, None, None, a, 0, v)
        if lib.pdt_conv_nt(*args) != 0:
            continue
        best = float("inf")
        for _ in range(3):
            ev0.record()
            for _ in range(3):
                lib.pdt_conv_nt(*args)
            ev1.record()
            ev1.synchronize()
            best = min(best, ev0.elapsed_time(ev1) / 3 * 1e3)
        res.append((best, v))
    res.sort()
    print(f"GEMM {n}^3 random bf16: " + " ".join(f"v{v}:{2.0 * n ** 3 / t / 1e6:.0f}TF" for t, v in res), flush=True)


if __name__ == "__main__":
    square()
    main()

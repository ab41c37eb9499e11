"""Per-shape microbenchmark: native HIP conv fwd / dgrad / wgrad vs the stock
MIOpen path (torch.nn.functional.conv2d and its autograd grads) on the
ResNet-50 conv shapes at batch 256 (``--batch``). The 7x7 stem row
times the direct stem GEMM; the model itself runs it as a space-to-depth GEMM. Prints one line per
shape with times in microseconds and the native/stock ratio.
"""
import argparse
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

SHAPES = [  # Cin, H, Cout, k, s, count-in-resnet50
    (3, 224, 64, 7, 2, 1),
    (64, 56, 64, 1, 1, 1), (64, 56, 64, 3, 1, 3), (64, 56, 256, 1, 1, 4), (256, 56, 64, 1, 1, 2),
    (256, 56, 128, 1, 1, 1), (128, 56, 128, 3, 2, 1), (256, 56, 512, 1, 2, 1),
    (128, 28, 512, 1, 1, 4), (512, 28, 128, 1, 1, 3), (128, 28, 128, 3, 1, 3), (512, 28, 256, 1, 1, 1),
    (256, 28, 256, 3, 2, 1), (512, 28, 1024, 1, 2, 1),
    (256, 14, 1024, 1, 1, 6), (1024, 14, 256, 1, 1, 5), (256, 14, 256, 3, 1, 5), (1024, 14, 512, 1, 1, 1),
    (512, 14, 512, 3, 2, 1), (1024, 14, 2048, 1, 2, 1),
    (512, 7, 2048, 1, 1, 3), (2048, 7, 512, 1, 1, 2), (512, 7, 512, 3, 1, 2),
]


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    N = a.batch
    tot = {"nf": 0, "nf0": 0, "sf": 0, "nd": 0, "sd": 0, "nw": 0, "sw": 0}
    print(f"{'shape':34s} {'fwd nat/stk us':>18s} {'dgrad nat/stk':>18s} {'wgrad nat/stk':>18s}  TFLOPs(fwd nat)")
    for Cin, H, Cout, k, s, cnt in SHAPES:
        p = k // 2
        conv = nn.Conv2d(Cin, Cout, k, s, p, bias=False).cuda().to(memory_format=torch.channels_last)
        x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        Cs = Cin if Cin % 8 == 0 else 8
        xs = x if Cs == Cin else F.pad(x.permute(0, 2, 3, 1), (0, Cs - Cin)).permute(0, 3, 1, 2).contiguous(
            memory_format=torch.channels_last)
        g = no._fwd_geom(N, H, H, Cs, conv)
        wb = no.bf16_weight(conv.weight, pad_cin_to=Cs if Cs != Cin else None)
        wbt = conv.weight.detach().to(torch.bfloat16)
        nf = timeit(lambda: no._conv_forward(xs, wb, N, H, H, Cs, Cout, g, with_stats=True), a.iters)
        nf0 = timeit(lambda: no._conv_forward(xs, wb, N, H, H, Cs, Cout, g, with_stats=False), a.iters)
        sf = timeit(lambda: F.conv2d(x, wbt, None, s, p), a.iters)
        y = F.conv2d(x, wbt, None, s, p)
        dy = torch.randn_like(y)
        w32 = conv.weight.detach().float()
        if Cin % 8 == 0:
            nd = timeit(lambda: no._conv_dgrad(dy, w32, N, H, H, Cs, Cout, g), a.iters)
            sd = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, wbt, None, (s, s), (p, p), (1, 1), False,
                                                                   (0, 0), 1, (True, False, False)), a.iters)
        else:
            nd = sd = 0.0
        dw = torch.empty((Cout, Cs, k, k), device="cuda", memory_format=torch.channels_last)
        nw = timeit(lambda: no._conv_wgrad(dy, xs, N, H, H, Cs, Cout, g, dw), a.iters)
        sw = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, wbt, None, (s, s), (p, p), (1, 1), False,
                                                               (0, 0), 1, (False, True, False)), a.iters)
        flop = 2.0 * N * g["Ho"] * g["Wo"] * Cout * Cin * k * k
        # roofline floor per pass: max(FLOP / 2.5 PF/s dense bf16, min bytes / 6 TB/s achievable HBM)
        bx, by, bw = 2.0 * N * H * H * Cs, 2.0 * N * g["Ho"] * g["Wo"] * Cout, 2.0 * Cout * Cs * k * k
        floor = lambda b: max(flop / 2.5e15, b / 6e12) * 1e6  # noqa: E731
        ff, fd, fw = floor(bx + by + bw), floor(bx + by + bw), floor(bx + by + 2 * bw)
        print(f"{Cin:4d}x{H:3d}->{Cout:4d} k{k} s{s} x{cnt:<2d}        {nf:8.1f}/{sf:8.1f} {nd:8.1f}/{sd:8.1f} "
              f"{nw:8.1f}/{sw:8.1f}  {flop / nf / 1e6:7.1f}  floor f/d/w {ff:6.1f}/{fd:6.1f}/{fw:6.1f} us"
              f"  eff {ff / nf:4.0%}/{(f'{fd / nd:4.0%}' if nd else '   -')}/{fw / nw:4.0%}", flush=True)
        for key, v in (("ff", ff), ("fd", fd), ("fw", fw)):
            tot[key] = tot.get(key, 0.0) + v * cnt
        print(f"{'':34s} fwd without the BN-statistics epilogue: {nf0:8.1f} us", flush=True)
        for key, v in (("nf", nf), ("nf0", nf0), ("sf", sf), ("nd", nd), ("sd", sd), ("nw", nw), ("sw", sw)):
            tot[key] += v * cnt
    print("weighted fwd total without statistics (ms): native %.2f vs stock %.2f" % (tot["nf0"] / 1e3, tot["sf"] / 1e3))
    print("weighted totals (ms, per ResNet-50 step): fwd %.2f/%.2f dgrad %.2f/%.2f wgrad %.2f/%.2f" % (
        tot["nf"] / 1e3, tot["sf"] / 1e3, tot["nd"] / 1e3, tot["sd"] / 1e3, tot["nw"] / 1e3, tot["sw"] / 1e3))
    print("roofline floors (ms): fwd %.2f dgrad %.2f wgrad %.2f" % (tot["ff"] / 1e3, tot["fd"] / 1e3,
                                                                    tot["fw"] / 1e3))


if __name__ == "__main__":
    main()

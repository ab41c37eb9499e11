"""How close the ResNet-50 bs-2048 1x1 weight gradients (csrc/conv_wgrad.hip, the tuned tile of
each shape's shipped table key) run to their floors.

For each shape: dW[Cout, Cin] = sum over the M = N*H*W pixels of dY[m, Cout] X[m, Cin]; the
bytes it must move (dY and X once, the fp32 split-K slabs written and reduced) against a
streaming reference measured on the same box (``torch.add``: 2 reads + 1 write), and the FLOPs
against a 1.3 PF/s bf16 MFMA rate (what the dense ring reaches at 8192^3). Prints one line per
shape with the time, TB/s, TF/s and the larger of the two floors.

    python scripts/wgrad_roofline.py [--batch 2048]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

# (H, Cin, Cout): the stride-1 1x1 convolutions of a ResNet-50 step (conv1 / conv3 of every
# bottleneck and the stage-1 downsample)
SHAPES = [(56, 64, 64), (56, 256, 64), (56, 64, 256), (28, 512, 128), (28, 128, 512), (14, 1024, 256),
          (14, 256, 1024), (7, 2048, 512), (7, 512, 2048)]
MFMA_RATE = 1.3e15


def timeit(fn, reps=5, rounds=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return statistics.median(ts) * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    torch.manual_seed(0)
    ref_a = torch.randn(256 << 20, device="cuda").to(torch.bfloat16)
    ref_b = torch.randn_like(ref_a)
    ref_o = torch.empty_like(ref_a)
    t_ref = timeit(lambda: torch.add(ref_a, ref_b, out=ref_o))
    stream = 3 * ref_a.numel() * 2 / t_ref
    print(f"stream reference {stream / 1e12:.2f} TB/s", flush=True)
    del ref_a, ref_b, ref_o
    tot_t = tot_f = 0.0
    for H, Cin, Cout in SHAPES:
        M = a.batch * H * H
        dy = (torch.randn(M, Cout, device="cuda") * 0.1).to(torch.bfloat16)
        x = torch.randn(M, Cin, device="cuda").to(torch.bfloat16)
        out = torch.empty(Cout, Cin, device="cuda")
        g = dict(M=M, Mo=Cout, No=Cin, ldy=Cout, Hs=H, Ws=H, C=Cin, Hm=H, Wm=H, sh=1, sw=1, oh0=0, ow0=0, dh=1,
                 dw=1, ntw=1)
        t = timeit(lambda: no.conv_wgrad(dy, x, out, **g))
        nbytes = M * (Cin + Cout) * 2
        flops = 2.0 * M * Cin * Cout
        floor = max(nbytes / stream, flops / MFMA_RATE)
        tot_t += t
        tot_f += floor
        print(f"H{H:3d} Cin {Cin:5d} Cout {Cout:5d}: {t * 1e6:8.1f} us  {nbytes / t / 1e12:5.2f} TB/s  "
              f"{flops / t / 1e12:6.0f} TF/s  floor {floor * 1e6:7.1f} us ({'bytes' if nbytes / stream > flops / MFMA_RATE else 'MFMA'})"
              f"  {floor / t * 100:5.1f} % of floor", flush=True)
        del dy, x, out
        torch.cuda.empty_cache()
    print(f"sum: {tot_t * 1e3:.2f} ms, floors {tot_f * 1e3:.2f} ms (one call per shape)")


if __name__ == "__main__":
    main()

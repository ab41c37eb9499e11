"""A/B of the attention kernels at the ViT-B/16 shape (B=256, T=197, H=12, d=64),
interleaved rounds in one process, median per arm:

  forward : whole-sequence 16x16 kernel (csrc/attention.hip) vs the 32x32-tile kernel
            (csrc/attention_f8.hip, bf16 scores) vs its fp8-score instantiation
  backward: dK/dV + dQ kernels with separate row + transposed LDS images vs one image

    python scripts/bench_attn.py [--batch 256] [--rounds 8]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--T", type=int, default=197)
ap.add_argument("--H", type=int, default=12)
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()
lib = no._load()
B, T, H = a.batch, a.T, a.H
dev = torch.device("cuda")
qkv = (torch.randn(B, T, 3 * H * 64, device=dev) * 1.5).to(torch.bfloat16)
out = torch.empty(B, T, H * 64, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B * H, T, dtype=torch.float32, device=dev)
dout = torch.randn(B, T, H * 64, device=dev).to(torch.bfloat16)
delta = torch.empty_like(lse)
dqkv = torch.empty_like(qkv)
P, st, sc = no._p, no._s(), 64 ** -0.5
arms = {
    "fwd seq16 (attention.hip)": lambda: lib.pdt_attn_fwd(P(qkv), P(out), P(lse), B, T, H, sc, st),
    "fwd tiles32 bf16": lambda: lib.pdt_attn_fwd_tiles(P(qkv), P(out), P(lse), B, T, H, sc, st),
    "fwd tiles32 fp8": lambda: lib.pdt_attn_fwd_f8(P(qkv), P(out), P(lse), B, T, H, sc, st),
}


def bwd(single):
    def f():
        lib.pdt_attn_set_bwd_single(single)
        return lib.pdt_attn_bwd(P(qkv), P(out), P(dout), P(lse), P(delta), P(dqkv), B, T, H, sc, st)
    return f


arms["bwd two images"] = bwd(0)
arms["bwd one image"] = bwd(1)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
times = {k: [] for k in arms}
lib.pdt_attn_fwd(P(qkv), P(out), P(lse), B, T, H, sc, st)
for r in range(a.rounds):
    for k, fn in arms.items():
        assert fn() == 0, k
        ev0.record()
        for _ in range(5):
            fn()
        ev1.record()
        ev1.synchronize()
        times[k].append(ev0.elapsed_time(ev1) / 5)
fl_fwd = 4 * B * H * T * T * 64
print(f"B={B} T={T} H={H}")
for k, t in times.items():
    med = statistics.median(t)
    fl = fl_fwd * (2.5 if k.startswith("bwd") else 1)
    print(f"{k:28s} median {med * 1e3:8.1f} us  min {min(t) * 1e3:8.1f} us  {fl / med / 1e9:6.1f} TFLOP/s")

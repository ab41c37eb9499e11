"""Time the fp8 attention kernels at the ViT-B/16 shape (B images, T = 197, H = 12, d = 64):
forward (pdt_attn_fwd_f8) and the fused backward (pdt_attn_bwd_f8), median of interleaved rounds.
Run it once per library build for an A/B (PDT_LIB_PATH selects the build).

    python scripts/bench_attn_f8.py [--batch 1024] [--rounds 10]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--T", type=int, default=197)
ap.add_argument("--H", type=int, default=12)
ap.add_argument("--rounds", type=int, default=10)
a = ap.parse_args()
lib = no._load()
B, T, H = a.batch, a.T, a.H
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
qkv = (torch.randn(B, T, 3 * H * 64, device=dev, generator=g) * 1.5).to(torch.bfloat16)
out = torch.empty(B, T, H * 64, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B * H, T, dtype=torch.float32, device=dev)
dout = torch.randn(B, T, H * 64, device=dev, generator=g).to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
P, st, sc = no._p, no._s(), 64 ** -0.5
# the ViT step's forward: the same kernel that also writes the e4m3 codes of O for the
# projection GEMM and rolls that GEMM's amax history (pdt_attn_fwd_f8_q8)
codes = torch.empty(B * T, H * 64, dtype=torch.uint8, device=dev)
meta = torch.zeros(lib.pdt_fp8_meta_words(), dtype=torch.float32, device=dev)
meta[0] = 1.0
part = torch.empty(B * H + 1, dtype=torch.float32, device=dev)
arms = {
    "fwd f8": lambda: lib.pdt_attn_fwd_f8(P(qkv), P(out), P(lse), B, T, H, sc, st),
    "fwd q8": lambda: lib.pdt_attn_fwd_f8_q8(P(qkv), P(out), P(lse), B, T, H, sc, P(codes), P(meta), P(part),
                                             P(part[-1:]), st),
    "bwd f8": lambda: lib.pdt_attn_bwd_f8(P(qkv), P(out), P(dout), P(lse), P(dqkv), B, T, H, sc, st),
}
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
times = {k: [] for k in arms}
assert arms["fwd f8"]() == 0
for r in range(a.rounds):
    for k, fn in arms.items():
        assert fn() == 0, k
        ev0.record()
        for _ in range(5):
            fn()
        ev1.record()
        ev1.synchronize()
        times[k].append(ev0.elapsed_time(ev1) / 5)
# a checksum of the gradient, so two builds can be compared for equal results
print(f"lib={os.environ.get('PDT_LIB_PATH', 'in-tree')} B={B} T={T} H={H} dqkv_sum={dqkv.float().abs().sum().item():.6e}")
for k, t in times.items():
    print(f"{k:8s} median {statistics.median(t) * 1e3:8.1f} us  min {min(t) * 1e3:8.1f} us")

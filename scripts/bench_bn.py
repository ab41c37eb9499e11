"""A/B of the BatchNorm element passes (csrc/bn_act.hip) at ResNet-50 stage-1
geometry, bs 1024 (M = 1024*56*56 rows, C = 256): trip unroll U = 1 / 2 / 4,
interleaved rounds in one process (guide §5.4 rule 24), median per arm, and the
achieved HBM bandwidth from the bytes each pass must move.

    python scripts/bench_bn.py [--batch 1024] [--rounds 8]
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
ap.add_argument("--C", type=int, default=256)
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()
lib = no._load()
dev = torch.device("cuda")
M, C = a.batch * 56 * 56, a.C
n = M * C
y = torch.randn(n, device=dev).to(torch.bfloat16)
res = torch.randn(n, device=dev).to(torch.bfloat16)
out = torch.empty_like(y)
dA = torch.randn(n, device=dev).to(torch.bfloat16)
dy = torch.empty_like(y)
mask = torch.empty(n // 8, dtype=torch.uint8, device=dev)
sc = torch.rand(C, device=dev) + 0.5
sh = torch.randn(C, device=dev) * 0.1
k1, k2, k3 = torch.randn(C, device=dev), torch.randn(C, device=dev) * 1e-3, torch.randn(C, device=dev) * 1e-3
st = no._s()
P = no._p


def apply():
    no._chk(lib.pdt_bn_apply(P(y), P(res), P(out), P(sc), P(sh), M, C, 1, P(mask), st), "apply")


def bwd_apply():
    no._chk(lib.pdt_bn_bwd_apply(P(dA), P(y), None, P(sc), P(sh), P(k1), P(k2), P(k3), P(dy), None, M, C, 1,
                                 P(mask), st), "bwd_apply")


passes = {"bn_apply res+relu+mask": (apply, n * 2 * 3 + n // 8),
          "bn_bwd_apply mask": (bwd_apply, n * 2 * 3 + n // 8)}
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
MODES = (1, 11, 2)  # 1 / 2: trip unroll; 11: unroll 1 + nontemporal stores
times = {(k, u): [] for k in passes for u in MODES}
for r in range(a.rounds):
    for u in MODES:
        assert lib.pdt_bn_set_unroll(u) == 0

        for k, (fn, _) in passes.items():
            fn()
            ev0.record()
            for _ in range(5):
                fn()
            ev1.record()
            ev1.synchronize()
            times[(k, u)].append(ev0.elapsed_time(ev1) / 5)
print(f"M={M} C={C} ({n * 2 / 2**30:.2f} GiB per bf16 tensor)")
for k, (_, nbytes) in passes.items():
    for u in MODES:
        t = times[(k, u)]
        med = statistics.median(t)
        print(f"{k:26s} mode={u:2d}: median {med * 1e3:8.1f} us  min {min(t) * 1e3:8.1f} us  {nbytes / med / 1e9:6.2f} TB/s")

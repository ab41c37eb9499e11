"""Do the BatchNorm element passes lose HBM bandwidth to address aliasing between their
streams? All activations come from the caching allocator at large-page-aligned bases,
so y[i], res[i] and out[i] share every low address bit. This times bn_apply (2 reads
+ 1 write + mask) and bn_bwd_apply at ResNet-50 stage 1, bs 1024 with the three
tensors as views at different byte offsets into larger buffers, plus a torch copy
(1R1W) for calibration. Interleaved rounds, median.

    python scripts/bench_bn_offsets.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

lib = no._load()
dev = torch.device("cuda")
M, C = 1024 * 56 * 56, 256
n = M * C
PAD = 8 << 20  # bytes of slack per buffer


def view_at(buf, off_bytes):
    return buf[off_bytes // 2: off_bytes // 2 + n]


bufs = [torch.empty(n + PAD // 2, dtype=torch.bfloat16, device=dev) for _ in range(4)]
for b in bufs:
    b.normal_()
mask = torch.empty(n // 8, dtype=torch.uint8, device=dev)
sc = torch.rand(C, device=dev) + 0.5
sh = torch.randn(C, device=dev) * 0.1
k1, k2, k3 = torch.randn(C, device=dev), torch.randn(C, device=dev) * 1e-3, torch.randn(C, device=dev) * 1e-3
st, P = no._s(), no._p
layouts = {  # byte offsets of (y, res/dA, out)
    "aligned": (0, 0, 0),
    "+0/+4K/+8K": (0, 4096, 8192),
    "+0/+64K/+128K": (0, 65536, 131072),
    "+0/+1M/+2M+4K": (0, 1 << 20, (2 << 20) + 4096),
    "+0/+2K/+5K": (0, 2048, 5120),
}
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
times = {}
for r in range(6):
    for name, (oy, orr, oo) in layouts.items():
        y, res, out = view_at(bufs[0], oy), view_at(bufs[1], orr), view_at(bufs[2], oo)
        arms = {
            f"apply {name}": lambda: lib.pdt_bn_apply(P(y), P(res), P(out), P(sc), P(sh), M, C, 1, P(mask), st),
            f"bwd_apply {name}": lambda: lib.pdt_bn_bwd_apply(P(res), P(y), None, P(sc), P(sh), P(k1), P(k2), P(k3),
                                                              P(out), None, M, C, 1, P(mask), st),
            f"copy {name}": lambda: out.copy_(y),
        }
        for k, fn in arms.items():
            fn()
            ev0.record()
            for _ in range(5):
                fn()
            ev1.record()
            ev1.synchronize()
            times.setdefault(k, []).append(ev0.elapsed_time(ev1) / 5)
for k, t in times.items():
    med = statistics.median(t)
    nb = n * 2 * (2 if k.startswith("copy") else 3) + (0 if k.startswith("copy") else n // 8)
    print(f"{k:32s} median {med * 1e3:8.1f} us  {nb / med / 1e9:6.2f} TB/s")

"""Time pdt_ln_bwd_f8_db (LayerNorm backward + residual gradient + e5m2 codes of dx + the producer's
bias column sums) at the ViT-B/16 bs1024 shape; PDT_LN_BWD_MAXB caps the block count (A/B).

    PDT_LN_BWD_MAXB=512 python scripts/bench_ln_bwd.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

lib = no._load()
rows, D = 201728, 768
dev = "cuda"
dy = torch.randn(rows, D, device=dev).to(torch.bfloat16)
x = torch.randn(rows, D, device=dev).to(torch.bfloat16)
add = torch.randn(rows, D, device=dev).to(torch.bfloat16)
g = torch.rand(D, device=dev) + 0.5
mean = x.float().mean(1)
rstd = torch.rsqrt(x.float().var(1, unbiased=False) + 1e-6)
_, _, gmeta = no.quantize_fp8_delayed(dy, None, no.E5M2)
blocks = lib.pdt_ln_bwd_blocks(rows)
dx = torch.empty_like(x)
part = torch.empty(2 * blocks * D, dtype=torch.float32, device=dev)
dg = torch.empty(D, dtype=torch.float32, device=dev)
db = torch.empty(D, dtype=torch.float32, device=dev)
codes = torch.empty(rows, D, dtype=torch.uint8, device=dev)
qpart = torch.empty(blocks + 1, dtype=torch.float32, device=dev)
cpart = torch.empty(blocks * D + lib.pdt_reduce_rows_work(blocks, D), dtype=torch.float32, device=dev)
pdb = torch.empty(D, dtype=torch.float32, device=dev)


def run():
    return lib.pdt_ln_bwd_f8_db(no._p(dy), no._p(x), no._p(g), no._p(mean), no._p(rstd), no._p(dx), no._p(dg),
                                no._p(db), no._p(part), rows, D, 0, no._p(add), no._p(codes), no._p(gmeta),
                                no._p(qpart), no._p(qpart[-1:]), no._p(cpart), no._p(pdb), 0, no._s())


assert run() == 0
torch.cuda.synchronize()
# dgamma / dbeta / bias sums against fp32 (the block count changes only their summation order)
xh = (x.float() - mean[:, None]) * rstd[:, None]
dyf = dy.float()
e_dg = ((dg - (dyf * xh).sum(0)).norm() / (dyf * xh).sum(0).norm()).item()
e_db = ((db - dyf.sum(0)).norm() / dyf.sum(0).norm()).item()
e_pdb = ((pdb - dx.float().sum(0)).norm() / dx.float().sum(0).norm()).item()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for _ in range(5):
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1) / 10)
gb = rows * D * (2 * 4 + 1) / 1e9  # dy, x, addend read + dx written (bf16), codes written
print(f"MAXB={os.environ.get('PDT_LN_BWD_MAXB', '512')} blocks={blocks} {rows}x{D}: {best * 1e3:7.1f} us "
      f"{gb / best:6.2f} TB/s  rel err dg {e_dg:.1e} db {e_db:.1e} bias {e_pdb:.1e}", flush=True)

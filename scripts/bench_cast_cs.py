"""Time pdt_cast_fp8_delayed_cs (bf16 -> e5m2 codes + column sums) at the ViT-B/16 bs1024 gradient
shapes; PDT_CAST_CS_RG=1 selects the previous one-walker-per-chunk block shape (A/B).

    python scripts/bench_cast_cs.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

lib = no._load()
for rows, cols in ((201728, 768), (201728, 2304), (201728, 3072)):
    x = torch.randn(rows, cols, device="cuda").to(torch.bfloat16)
    _, _, meta = no.quantize_fp8_delayed(x, None, no.E5M2)
    nb = lib.pdt_cast_cs_bands(rows)
    cpart = torch.empty(nb * cols + lib.pdt_reduce_rows_work(nb, cols), dtype=torch.float32, device="cuda")
    q = torch.empty(rows, cols, dtype=torch.uint8, device="cuda")
    dq = torch.empty(1, dtype=torch.float32, device="cuda")
    db = torch.empty(cols, dtype=torch.float32, device="cuda")

    def run():
        return lib.pdt_cast_fp8_delayed_cs(no._p(x), rows, cols, no._p(meta), no.E5M2, no._p(q), no._p(dq),
                                           no._p(cpart), no._p(db), no._s())
    assert run() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10)
    gb = rows * cols * 3 / 1e9  # bf16 read + e5m2 write
    print(f"RG={os.environ.get('PDT_CAST_CS_RG', 'auto')} {rows}x{cols}: {best * 1e3:7.1f} us  {gb / best:6.2f} TB/s",
          flush=True)

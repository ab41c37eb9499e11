"""Host enqueue cost of one bench training step, split by phase, with the GPU idle.

    python scripts/host_split.py [--model resnet50] [--batch 256] [--reps 5]

Each phase (batch fetch, forward, backward, optimizer) is timed on the host after a
``torch.cuda.synchronize()``, so the submission queue never throttles the host: the
numbers are the pure Python + launch cost the step pays per iteration.
Reports the median over ``--reps`` steps after warm-up."""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd import models  # noqa: E402
from pytorch_distributed_template_amd.data.synthetic import SyntheticImageNetLoader  # noqa: E402
from pytorch_distributed_template_amd.ops import fused  # noqa: E402
from pytorch_distributed_template_amd.optim import FusedSGD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--set", action="append", default=[], metavar="K=V")
    a = ap.parse_args()
    for kv in a.set:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    fused.set_backend("native")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = getattr(models, a.model)(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    loader = SyntheticImageNetLoader(a.batch, num_samples=a.batch * 64, dtype="bfloat16", device=dev)
    it = iter(loader)
    rows = []
    for i in range(3 + a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x, y = next(it)
        t1 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss = fused.softmax_cross_entropy(model(x), y)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        opt.step()
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        if i >= 3:
            rows.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0, t5 - t0))
    med = [statistics.median(r[k] for r in rows) * 1e3 for k in range(6)]
    print(f"{a.model} bs {a.batch}: host ms  batch {med[0]:.2f}  forward {med[1]:.2f}  backward {med[2]:.2f}  "
          f"optimizer {med[3]:.2f}  total enqueue {med[4]:.2f}  | enqueue+drain {med[5]:.2f}", flush=True)


if __name__ == "__main__":
    main()

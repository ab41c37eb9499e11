"""The reference's own model on its own config shape: MnistModel (LeNet, 21,840 params),
batch 128 of [1, 28, 28], NLL loss, Adam(lr=1e-3, amsgrad=True) -- one training step =
forward + loss + backward + optimizer step, timed on device (HIP events) for the native
kernels (csrc/lenet.hip + fused Adam) and for the stock PyTorch-ROCm ops
(MIOpen / rocBLAS + torch.optim.Adam), on synthetic MNIST-shaped data.

    python scripts/lenet_bench.py [--batch 128] [--steps 200]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.models.loss import nll_loss  # noqa: E402
from pytorch_distributed_template_amd.models.mnist import MnistModel  # noqa: E402
from pytorch_distributed_template_amd.ops import fused  # noqa: E402
from pytorch_distributed_template_amd.optim import FusedAdam  # noqa: E402


def run(backend, batch, steps, warmup=20):
    torch.manual_seed(0)
    fused.set_backend(backend)
    dev = torch.device("cuda", 0)
    m = MnistModel().to(dev).train()
    if backend == "native":
        opt = FusedAdam(m.parameters(), lr=1e-3, amsgrad=True)
    else:
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, amsgrad=True)
    g = torch.Generator(device=dev).manual_seed(1)
    xs = [torch.rand(batch, 1, 28, 28, device=dev, generator=g) for _ in range(4)]
    ys = [torch.randint(0, 10, (batch,), device=dev, generator=g) for _ in range(4)]

    def step(i):
        opt.zero_grad(set_to_none=True)
        loss = nll_loss(m(xs[i % 4]), ys[i % 4])  # the config's loss (native NLL kernel on GPU)
        loss.backward()
        opt.step()
        return loss

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for i in range(steps):
        loss = step(i)
    e1.record()
    e1.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    fused.set_backend("auto")
    return {"backend": backend, "batch": batch, "ms_per_step": round(e0.elapsed_time(e1) / steps, 4),
            "wall_ms_per_step": round(wall, 4), "img_per_s": round(batch * steps / (e0.elapsed_time(e1) / 1e3), 1),
            "final_loss": round(float(loss), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    for backend in ("native", "torch"):
        print(json.dumps(run(backend, a.batch, a.steps)), flush=True)


if __name__ == "__main__":
    main()

"""Time one fused optimizer step (FusedSGD on ResNet-50's parameters, FusedAdam(amsgrad) on
LeNet's) for several work-list chunk sizes (optim/fused.py CHUNK).

    python scripts/bench_optim.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd import models  # noqa: E402
from pytorch_distributed_template_amd.optim import FusedAdam, FusedSGD  # noqa: E402
from pytorch_distributed_template_amd.optim import fused as F  # noqa: E402


def timed(opt, n=50):
    for _ in range(5):
        opt.step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        opt.step()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    r50 = models.resnet50(num_classes=1000).cuda().to(memory_format=torch.channels_last)
    lenet = models.MnistModel().cuda()
    for m in (r50, lenet):
        for p in m.parameters():
            p.grad = torch.randn_like(p) * 1e-3
    n50 = sum(p.numel() for p in r50.parameters())
    for chunk in (65536, 32768, 16384, 8192, 4096):
        F.CHUNK = chunk
        t1 = timed(FusedSGD(r50.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5))
        t2 = timed(FusedAdam(lenet.parameters(), lr=1e-3, amsgrad=True, write_bf16_shadow=False))
        gbs = n50 * 22 / (t1 * 1e-6) / 1e9
        print(f"CHUNK {chunk:6d}: ResNet-50 FusedSGD {t1:7.1f} us ({gbs:5.0f} GB/s)  LeNet FusedAdam {t2:6.1f} us",
              flush=True)


if __name__ == "__main__":
    main()

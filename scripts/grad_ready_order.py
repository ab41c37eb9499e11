"""When does each DDP gradient bucket become ready during the native backward?

Runs ResNet-50 / ResNet-152 (native kernels, bf16) forward + backward on one GPU
with a post-accumulate-grad hook on every parameter. Each hook records a HIP
event on the current stream, so the time a gradient is READY ON THE DEVICE is
known (host-side hook times would only say when the kernels were queued). The
parameters are grouped into buckets exactly as DDP would build them
(``parallel.ddp.bucket_plan``: reverse registration order, 1 MiB first bucket,
``--bucket-mb`` cap) and the script prints, per bucket, when its last gradient
was ready relative to the start and the end of backward: the time that bucket's
all-reduce has to hide behind the remaining backward.

    python scripts/grad_ready_order.py [--model resnet50] [--batch 256] [--bucket-mb 64]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_template_amd import models  # noqa: E402
from pytorch_distributed_template_amd.ops import fused, native_ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet50")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--bucket-mb", type=float, default=64.0)
ap.add_argument("--grad-bytes", type=int, default=4, help="4: fp32 buckets, 2: bf16-compressed")
a = ap.parse_args()

native_ops.require()
fused.set_backend("native")
dev = torch.device("cuda")
torch.manual_seed(0)
model = getattr(models, a.model)(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
x = native_ops.synthetic_images((a.batch, 3, 224, 224), torch.bfloat16, dev, seed=1)
y = torch.randint(0, 1000, (a.batch,), device=dev)
names = {id(p): n for n, p in model.named_parameters()}
params = [p for p in model.parameters() if p.requires_grad]

# DDP's bucket assignment (reverse registration order; first bucket capped at 1 MiB)
rev = list(reversed(params))
import torch.distributed as dist  # noqa: E402
idx, _ = dist._compute_bucket_assignment_by_size(rev, [1024 * 1024, int(a.bucket_mb * 2 ** 20)])
bucket_of = {}
for b, ids in enumerate(idx):
    for i in ids:
        bucket_of[id(rev[i])] = b

events = {}


def hook(p):
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    events[id(p)] = ev


for p in params:
    p.register_post_accumulate_grad_hook(hook)

for it in range(3):  # warm (autotune), then measure the last iteration
    events.clear()
    model.zero_grad(set_to_none=True)
    loss = fused.softmax_cross_entropy(model(x), y)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    loss.backward()
    t1.record()
    torch.cuda.synchronize()

bwd_ms = t0.elapsed_time(t1)
ready = sorted(((t0.elapsed_time(events[id(p)]), names[id(p)], bucket_of[id(p)], p.numel()) for p in params))
print(f"{a.model} bs{a.batch}: backward {bwd_ms:.2f} ms, {len(params)} parameter tensors, "
      f"{len(idx)} buckets (cap {a.bucket_mb} MiB, {a.grad_bytes}-byte grads)")
print("\nper bucket: size, last gradient ready (ms after backward start), backward left to hide its all-reduce")
for b in range(len(idx)):
    ts = [t for t, _, bb, _ in ready if bb == b]
    nbytes = sum(rev[i].numel() for i in idx[b]) * a.grad_bytes
    print(f"  bucket {b}: {nbytes / 2**20:7.2f} MiB  ready at {max(ts):7.2f} ms  hides behind {bwd_ms - max(ts):7.2f} ms")
print("\nreadiness order (first / last 12 tensors):")
for row in (ready[:12] + ready[-12:]) if len(ready) > 24 else ready:
    t, n, b, k = row
    print(f"  {t:8.2f} ms  bucket {b}  {n} ({k})")

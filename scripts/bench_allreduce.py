"""RCCL all-reduce bandwidth sweep (rccl-tests is not installed in this image).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        scripts/bench_allreduce.py [--dtype bf16|fp32] [--min-mb 1] [--max-mb 512]

Prints, per message size, the time, algorithm bandwidth (bytes / time) and
bus bandwidth (algbw * 2(n-1)/n: the per-link rate a ring achieves, to compare
against the ~153 GB/s of one xGMI link and 7 links per MI355X). Use it to pick
DDP ``bucket_cap_mb``: the smallest size that reaches the plateau.
"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--min-mb", type=float, default=1)
    ap.add_argument("--max-mb", type=float, default=512)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pytorch_distributed_template_amd.utils.dist import init_distributed
    dev = init_distributed()
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    esz = torch.tensor([], dtype=dt).element_size()
    mb = a.min_mb
    if rank == 0:
        print(f"world={world} dtype={a.dtype}")
        print(f"{'size_MB':>10s} {'time_us':>10s} {'algbw_GB/s':>11s} {'busbw_GB/s':>11s}")
    while mb <= a.max_mb:
        n = int(mb * 2 ** 20 / esz)
        t = torch.ones(n, dtype=dt, device=dev)
        for _ in range(3):
            if world > 1:
                dist.all_reduce(t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            if world > 1:
                dist.all_reduce(t)
        torch.cuda.synchronize()
        dt_s = (time.perf_counter() - t0) / a.iters
        alg = n * esz / dt_s / 1e9
        bus = alg * 2 * (world - 1) / max(world, 1)
        if rank == 0:
            print(f"{mb:10.1f} {dt_s * 1e6:10.1f} {alg:11.1f} {bus:11.1f}", flush=True)
        mb *= 2
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

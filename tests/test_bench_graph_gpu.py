"""bench.py's HIP-graph preflight (``graph_collectives_ok``) on a real RCCL group: capture one
all-reduce on a throwaway group, replay it, agree on the main group. On one GPU the group has
one rank (the N > 1 case runs the same code on the driver's multi-GPU node)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["PDT_ROOT"])
import bench
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
ok, why = bench.graph_collectives_ok(dev, 1, check_single=True)
print("RESULT", ok, why)
dist.destroy_process_group()
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_graph_collectives_preflight_one_rank():
    env = dict(os.environ, PDT_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               TORCH_NCCL_ASYNC_ERROR_HANDLING="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "RESULT True None" in r.stdout, (r.stdout, r.stderr[-2000:])

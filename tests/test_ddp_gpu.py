"""DDP over two ranks sharing the one GPU of the test box (gloo transport for
the gradient buckets; RCCL needs one GPU per rank), with the native HIP kernels
doing every forward/backward op. The DDP-averaged gradient must equal the mean
of the per-rank local gradients (BN statistics are per rank, as in DDP)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK="0")
        import torch.distributed as dist
        from pytorch_distributed_template_amd.models import resnet50
        from pytorch_distributed_template_amd.ops import fused
        from pytorch_distributed_template_amd.parallel import wrap_ddp
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
        fused.set_backend("native")
        torch.manual_seed(0)
        model = resnet50(num_classes=16).cuda().to(memory_format=torch.channels_last)
        ref = resnet50(num_classes=16).cuda().to(memory_format=torch.channels_last)
        ref.load_state_dict(model.state_dict())
        g = torch.Generator(device="cpu").manual_seed(100 + rank)
        x = torch.randn(4, 3, 64, 64, generator=g).cuda().to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 16, (4,), generator=g).cuda()
        # local gradient, then the explicit cross-rank mean
        fused.softmax_cross_entropy(ref(x), y).backward()
        local = [p.grad.detach().clone() for p in ref.parameters()]
        for t in local:
            dist.all_reduce(t)
            t /= world
        ddp = wrap_ddp(model, torch.device("cuda", 0), bucket_cap_mb=8, broadcast_buffers=False)
        fused.softmax_cross_entropy(ddp(x), y).backward()
        err = max(float((p.grad - t).abs().max() / t.abs().max().clamp_min(1e-6)) for p, t in
                  zip(model.parameters(), local))
        q.put((rank, err))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_ddp_two_ranks_native_kernels():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(60)
    for r, v in res.items():
        assert not isinstance(v, str), v
        assert v < 1e-3, (r, v)


def test_bench_two_gloo_ranks_native_kernels_reducer_in_sync():
    """bench.py at N = 2 on the one GPU: two ranks (gloo transport, RCCL needs a GPU per rank)
    running the native kernels and the framework's reducer for several optimizer steps; the
    JSON line must report a finite loss and ``ranks_in_sync`` (bitwise-equal weights)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--batch", "64", "--steps", "3", "--warmup", "1"], cwd=root, env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    c = rec["config"]
    assert rec["n_gpus"] == 2 and c["backend"] == "native" and c["ddp_impl"] == "BucketedDDP"
    assert c["loss_first"] is not None and c["loss_last"] is not None
    assert c["ranks_in_sync"] is True and c["ranks_checked"] == 2, c

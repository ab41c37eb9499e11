"""HIP-graph training steps (bench.py's default, ``trainer.hip_graph``):

* the fused optimizers in capturable mode, captured once in a HIP graph and replayed
  with an lr that changes between replays, follow torch.optim stepping eagerly
  (Adam's bias corrections advance on the device; ``state_dict`` reports the step);
* ``train.py`` with ``trainer.hip_graph`` (capture after the warm-up, replays, a
  scheduler changing the lr between epochs, checkpoint) ends at the same weights as
  the same run stepped eagerly.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _params(seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    shapes = [(64, 3, 7, 7), (1000, 2048), (1000,), (37,)]
    ps = []
    for s in shapes:
        t = torch.randn(s, device="cuda", generator=g)
        if t.dim() == 4:
            t = t.contiguous(memory_format=torch.channels_last)
        ps.append(torch.nn.Parameter(t))
    return ps


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw"])
def test_capturable_fused_optimizer_in_graph_matches_torch(kind):
    from pytorch_distributed_template_amd.optim import FusedAdam, FusedAdamW, FusedSGD
    pf, pr = _params(1), _params(1)
    if kind == "sgd":
        kw = dict(lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
        opt = FusedSGD(pf, capturable=True, **kw)
        ref = torch.optim.SGD(pr, **kw)
    else:
        kw = dict(lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.05, amsgrad=True)
        opt = (FusedAdam if kind == "adam" else FusedAdamW)(pf, capturable=True, **kw)
        ref = (torch.optim.Adam if kind == "adam" else torch.optim.AdamW)(pr, **kw)
    gen = torch.Generator(device="cuda").manual_seed(7)
    for p in pf:
        p.grad = torch.zeros_like(p)
    lrs = [kw["lr"], kw["lr"], kw["lr"] * 0.5, kw["lr"] * 0.5, kw["lr"] * 0.25, kw["lr"] * 0.125]

    def new_grads():
        return [torch.randn(p.shape, device="cuda", generator=gen) for p in pf]

    graph = None
    for i, lr in enumerate(lrs):
        gs = new_grads()
        for p, q, g in zip(pf, pr, gs):
            p.grad.copy_(g)
            q.grad = g.clone()
        for grp in opt.param_groups:
            grp["lr"] = lr
        for grp in ref.param_groups:
            grp["lr"] = lr
        ref.step()
        if i < 2:  # eager warm-up: state and device scalars exist before the capture
            opt.step()
            continue
        if graph is None:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side), torch.cuda.graph(graph, stream=side):
                opt.step()
            torch.cuda.current_stream().wait_stream(side)
        opt.refresh_scalars()
        graph.replay()
    torch.cuda.synchronize()
    for p, q in zip(pf, pr):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-5, atol=2e-6)
    if kind != "sgd":
        sd = opt.state_dict()
        assert all(float(st["step"]) == len(lrs) for st in sd["state"].values())


def test_trainer_hip_graph_matches_eager(tmp_path):
    base = json.loads((ROOT / "config" / "resnet50_bf16.json").read_text())
    base["trainer"].update(len_epoch=14, epochs=2, monitor="off", save_period=2)
    base["train_loader"]["args"].update(batch_size=16, num_samples=16 * 14)
    base["lr_scheduler"] = {"type": "StepLR", "args": {"step_size": 1, "gamma": 0.5}}
    weights = {}
    for mode in ("graph", "eager"):
        cfg = json.loads(json.dumps(base))
        cfg["trainer"].update(save_dir=str(tmp_path / mode), hip_graph=mode == "graph")
        p = tmp_path / f"{mode}.json"
        p.write_text(json.dumps(cfg))
        env = dict(os.environ, PYTHONPATH=str(ROOT), PDT_RUN_ID=mode)
        r = subprocess.run([sys.executable, "train.py", "-c", str(p), "--backend", "native", "--no-validate",
                            "--seed", "0", "--deterministic"], cwd=ROOT, env=env, capture_output=True, text=True,
                           timeout=900)
        out = r.stdout + r.stderr
        assert r.returncode == 0, out[-4000:]
        assert ("captured the training step as a HIP graph" in out) == (mode == "graph"), out[-3000:]
        ck = tmp_path / mode / cfg["name"] / "train" / mode / "checkpoint-epoch2.pth"
        state = torch.load(ck, weights_only=True, map_location="cpu")
        weights[mode] = state["state_dict"]
    for k, v in weights["eager"].items():
        if v.is_floating_point():
            torch.testing.assert_close(weights["graph"][k].float(), v.float(), rtol=1e-3, atol=1e-4, msg=k)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_trainer_hip_graph_under_torchrun_ddp_rccl(tmp_path):
    """``trainer.hip_graph`` with DDP over a 1-rank RCCL group (torchrun): the reducer is
    built on the capture side stream, the RCCL watchdog is drained before the capture, the
    captured step (bucketed all-reduce included) is replayed, a scheduler changes the lr
    between the epochs, checkpoints are written -- and the weights after 2 epochs equal those
    of the same torchrun job stepped eagerly (a gradient the reducer doubled or dropped in
    the captured step shows up here: the graph path keeps gradients across steps)."""
    base = json.loads((ROOT / "config" / "resnet50_bf16.json").read_text())
    base["trainer"].update(len_epoch=14, epochs=2, monitor="off", save_period=2)
    base["train_loader"]["args"].update(batch_size=16, num_samples=16 * 14)
    base["lr_scheduler"] = {"type": "StepLR", "args": {"step_size": 1, "gamma": 0.5}}
    for k in ("valid_loader", "test_loader"):
        base[k]["args"].update(batch_size=16, num_samples=32)
    weights = {}
    for mode in ("graph", "eager"):
        cfg = json.loads(json.dumps(base))
        cfg["trainer"].update(save_dir=str(tmp_path / mode), hip_graph=mode == "graph")
        p = tmp_path / f"{mode}.json"
        p.write_text(json.dumps(cfg))
        env = dict(os.environ, PYTHONPATH=str(ROOT), PDT_RUN_ID=mode, HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "train.py", "-c", str(p),
               "--backend", "native", "--seed", "0", "--deterministic"]
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
        out = r.stdout + r.stderr
        assert r.returncode == 0, out[-4000:]
        assert "process group: nccl, world size 1" in out, out[-3000:]
        assert ("captured the training step as a HIP graph" in out) == (mode == "graph"), out[-3000:]
        ck = tmp_path / mode / cfg["name"] / "train" / mode / "checkpoint-epoch2.pth"
        state = torch.load(ck, weights_only=True, map_location="cpu")
        assert abs(state["optimizer"]["param_groups"][0]["lr"] - 0.1 * 0.25) < 1e-9  # two StepLR steps
        weights[mode] = state["state_dict"]
    for k, v in weights["eager"].items():
        if v.is_floating_point():
            assert torch.isfinite(weights["graph"][k]).all(), k
            torch.testing.assert_close(weights["graph"][k].float(), v.float(), rtol=1e-3, atol=1e-4, msg=k)

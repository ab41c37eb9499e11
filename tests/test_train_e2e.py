"""End-to-end plumbing on CPU (BASELINE config #1: MNIST LeNet via config.json,
gloo): train -> checkpoint files/keys -> resume -> test.py; and a 2-rank
torchrun job writing ONE run dir."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
ENV = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2", PDT_RUN_ID="")


def _cfg(tmp_path, epochs=2, monitor="min val_loss"):
    cfg = json.loads((ROOT / "config" / "mnist_cpu.json").read_text())
    cfg["trainer"]["save_dir"] = str(tmp_path / "saved")
    cfg["trainer"]["epochs"] = epochs
    cfg["trainer"]["monitor"] = monitor
    cfg["trainer"]["tensorboard"] = True
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    return p


def _run(args, env_extra=None, timeout=300):
    env = dict(ENV)
    env.pop("PDT_RUN_ID")
    if env_extra:
        env.update(env_extra)
    r = subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout + r.stderr


def test_train_resume_test(tmp_path):
    cfg = _cfg(tmp_path)
    out = _run(["train.py", "-c", str(cfg), "--seed", "0", "--lr", "0.002"], {"PDT_RUN_ID": "run1"})
    run = tmp_path / "saved" / "Mnist_LeNet_cpu" / "train" / "run1"
    assert (run / "config.json").exists() and (run / "info.log").exists()
    assert (run / "checkpoint-epoch1.pth").exists() and (run / "checkpoint-epoch2.pth").exists()
    assert (run / "model_best.pth").exists()
    assert "Trainable parameters: 21840" in out
    assert "val_loss" in out and "val_accuracy" in out
    ck = torch.load(run / "checkpoint-epoch2.pth", weights_only=True)
    assert set(ck) >= {"arch", "epoch", "state_dict", "optimizer", "monitor_best", "config"}
    assert ck["arch"] == "MnistModel" and ck["epoch"] == 2
    assert ck["config"]["optimizer"]["args"]["lr"] == 0.002
    assert not any(k.startswith("module.") for k in ck["state_dict"])
    log = (run / "info.log").read_text()
    assert "    epoch          : 2" in log
    # val loss is real (reference Q1: it was always 0)
    assert "val_loss       : 0\n" not in log

    # resume: new run dir, continues at epoch 3
    _run(["train.py", "-r", str(run / "checkpoint-epoch2.pth"), "--epochs", "3"], {"PDT_RUN_ID": "run2"})
    run2 = tmp_path / "saved" / "Mnist_LeNet_cpu" / "train" / "run2"
    assert (run2 / "checkpoint-epoch3.pth").exists() and not (run2 / "checkpoint-epoch1.pth").exists()
    assert "Resume training from epoch 3" in (run2 / "info.log").read_text()

    # evaluation
    out = _run(["test.py", "-r", str(run2 / "checkpoint-epoch3.pth"), "--seed", "1"], {"PDT_RUN_ID": "t1"})
    assert "'loss':" in out and "'accuracy':" in out and "'top_k_acc':" in out
    assert (tmp_path / "saved" / "Mnist_LeNet_cpu" / "test" / "t1" / "info.log").exists()


def test_monitor_off_and_no_validate(tmp_path):
    cfg = _cfg(tmp_path, epochs=1, monitor="off")
    _run(["train.py", "-c", str(cfg), "--no-validate"], {"PDT_RUN_ID": "off"})
    run = tmp_path / "saved" / "Mnist_LeNet_cpu" / "train" / "off"
    assert (run / "checkpoint-epoch1.pth").exists() and not (run / "model_best.pth").exists()


def test_torchrun_two_ranks_gloo_single_run_dir(tmp_path):
    cfg = _cfg(tmp_path, epochs=1)
    _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr", "127.0.0.1",
          "--master-port", str(29500 + os.getpid() % 1000), "train.py", "-c", str(cfg)])
    runs = list((tmp_path / "saved" / "Mnist_LeNet_cpu" / "train").iterdir())
    assert len(runs) == 1, runs                      # reference Q5: one dir per rank
    assert (runs[0] / "checkpoint-epoch1.pth").exists()
    ck = torch.load(runs[0] / "checkpoint-epoch1.pth", weights_only=True)
    assert ck["arch"] == "MnistModel"


def test_legacy_local_rank_flag_accepted(tmp_path):
    cfg = _cfg(tmp_path, epochs=1, monitor="off")
    _run(["train.py", "-c", str(cfg), "--local-rank=0", "--no-validate"], {"PDT_RUN_ID": "lr1"})
    _run(["train.py", "-c", str(cfg), "--local_rank", "0", "--no-validate"], {"PDT_RUN_ID": "lr2"})


def test_tensorboard_loss_curve_per_log_step(tmp_path):
    """loss/train is written every log_step iterations (reference trainer.py:60-62 writes it
    every iteration), not once per epoch: 2048 synthetic images / batch 128 = 16 iterations,
    log_step = int(sqrt(128)) = 11 -> iterations 0 and 11 of each epoch."""
    cfg = _cfg(tmp_path, epochs=2, monitor="off")
    _run(["train.py", "-c", str(cfg), "--no-validate"], {"PDT_RUN_ID": "tb"})
    run = tmp_path / "saved" / "Mnist_LeNet_cpu" / "train" / "tb"
    recs = [json.loads(ln) for ln in (run / "scalars.jsonl").read_text().splitlines()]
    loss = [r for r in recs if r["tag"] == "loss/train"]
    assert [r["step"] for r in loss] == [0, 11, 16, 27], loss
    assert all(r["value"] > 0 for r in loss)

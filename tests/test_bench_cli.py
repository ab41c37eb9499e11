"""bench.py launcher contract (CPU): ``--gpus N`` must run N ranks or fail loudly.

The driver runs ``python bench.py --gpus N`` (and the torch.distributed.run
form); a silent 1-rank run reported as the N-GPU point would corrupt the
scaling curve (missing #1).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["OMP_NUM_THREADS"] = "2"
    return env


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_self_launches_two_cpu_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--device", "cpu", "--batch", "2", "--image-size", "32",
                        "--steps", "1", "--warmup", "1"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 4
    assert rec["config"]["dist_backend"] == "gloo"
    assert rec["steps"] == 1 and rec["warmup"] == 1
    assert rec["value"] > 0
    assert rec["config"]["ddp_impl"] == "BucketedDDP"  # the framework's reducer, not torch DDP
    assert rec["config"]["ranks_in_sync"] is True and rec["config"]["ranks_checked"] == 2


@pytest.mark.skipif(__import__("torch").cuda.device_count() >= 2, reason="host has >= 2 GPUs")
def test_bench_refuses_more_gpus_than_visible():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "GPU(s) are visible" in r.stderr
    assert '"metric"' not in r.stdout


def test_bench_rejects_world_size_mismatch():
    env = _env()
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--steps", "1", "--warmup", "0"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_bench_one_rank_runs_ddp_over_a_process_group():
    """N = 1 measures the same DDP path as N > 1: a 1-rank process group (gloo on
    the CPU rehearsal, RCCL on a GPU) and the DDP reducer; --no-ddp drops both."""
    base = [sys.executable, BENCH, "--gpus", "1", "--device", "cpu", "--batch", "2", "--image-size", "32",
            "--steps", "1", "--warmup", "1"]
    r = subprocess.run(base, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 1 and rec["config"]["dist_backend"] == "gloo" and rec["config"]["ddp"] is True
    r = subprocess.run(base + ["--no-ddp"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["config"]["ddp"] is False and rec["config"]["dist_backend"].startswith("none")


def test_bench_eight_cpu_ranks_one_json_line():
    """The driver's N = 8 launch, rehearsed on 8 gloo ranks: one JSON line from rank 0 with
    the whole-job numbers (dp8), finite first / last losses."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--device", "cpu", "--batch", "2", "--image-size", "32",
                        "--steps", "2", "--warmup", "1"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == "dp8"
    assert rec["config"]["global_batch"] == 16
    assert rec["config"]["loss_first"] is not None and rec["config"]["loss_last"] is not None
    assert rec["config"]["grad_allreduce_probe"] is None  # CPU ranks: no RCCL probe
    # the framework's reducer over 8 ranks, 3 optimizer steps: every rank holds the same weights
    assert rec["config"]["ddp_impl"] == "BucketedDDP"
    assert rec["config"]["ranks_in_sync"] is True and rec["config"]["ranks_checked"] == 8
    assert rec["config"]["param_checksum_max_rank_diff"] == 0.0


def test_bench_refuses_a_nan_step():
    """A diverged step (lr 1e30 -> NaN loss) is reported with value null and a non-zero exit,
    never as throughput."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--device", "cpu", "--batch", "2", "--image-size", "32",
                        "--steps", "2", "--warmup", "2", "--lr", "1e30"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    rec = _json_line(r.stdout)
    assert rec["value"] is None and rec["vs_baseline"] is None
    assert "non-finite" in rec["error"]
    assert rec["config"]["loss_last"] is None

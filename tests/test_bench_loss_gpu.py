"""bench.py rejects a broken step: a short ResNet-50 run at batch 256,
eager and ``--graph``, must report finite first / last losses; the graph run must also pass
its eager-vs-replay check (the same batches at lr 0 give the same losses)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "2", "--batch", "256"] + extra,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_eager_and_graph_losses_finite_and_agree():
    eager = _run([])
    graph = _run(["--graph"])
    for rec in (eager, graph):
        c = rec["config"]
        assert rec["value"] and rec["value"] > 0
        assert c["loss_first"] is not None and c["loss_last"] is not None
        assert 0.0 < c["loss_first"] < 20.0 and 0.0 < c["loss_last"] < 20.0
    gc = graph["config"]["graph_check"]
    assert graph["config"]["hip_graph"] is True and gc is not None
    assert gc["max_rel_diff"] <= 1e-3, gc
    # (no cross-run loss comparison: the graph run warms up 11 steps at lr 0.1 before its first
    # timed step, the eager run 2, so their first timed losses sit at different points of an
    # unstable random-label trajectory -- 7.25 vs 9.53 on one box. The same-batch agreement that
    # matters is graph_check above: eager and replayed steps from one state, lr 0.)

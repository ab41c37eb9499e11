"""Multi-process (gloo, world 2, 127.0.0.1) tests of the distributed layer:
collectives, sampler sharding, DDP gradient equivalence, single run dir."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from pytorch_distributed_template_amd.utils import dist as pdist
    dev = pdist.init_distributed(backend="gloo")
    assert dev.type == "cpu"
    return pdist


def _w_collectives(rank, world, port, q):
    try:
        pdist = _init(rank, world, port)
        out = {}
        out["rank"] = pdist.get_rank()
        # tensors leave the rank as lists: a tensor in the result queue travels as a shared fd that
        # the parent may try to fetch after this process has exited (EOFError under load)
        out["gather_obj"] = [{"r": d["r"], "t": d["t"].tolist()}
                             for d in pdist.all_gather({"r": rank, "t": torch.tensor([rank])})]
        t = torch.arange(rank + 2, dtype=torch.float32)  # variable length
        g = pdist.gather_tensors(t, dst=0)
        out["gather_t"] = None if g is None else [x.tolist() for x in g]
        out["reduce"] = float(pdist.reduce_loss(torch.tensor(float(rank + 1))))
        out["bcast"] = pdist.broadcast_object({"x": 5} if rank == 0 else None)
        out["mean"] = float(pdist.all_reduce_mean(torch.tensor(float(rank))))
        pdist.synchronize()
        q.put((rank, out))
        pdist.cleanup()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def _run_once(fn, world, extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=fn, args=(r, world, port, q) + extra) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=120) for _ in range(world))
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    return res


def _run(fn, world=2, *extra):
    # one retry with a fresh port: _free_port() releases the port before the ranks bind it,
    # so another process on the machine can take it in between (seen once under load)
    # -- retried ONLY for an address-in-use / bind failure; any other rank error is a real
    # failure and is reported from the first run
    res = _run_once(fn, world, extra)
    errs = [v for v in res.values() if isinstance(v, str)]
    if errs and all(("ddress already in use" in e or "EADDRINUSE" in e or "bind" in e.lower()) for e in errs):
        res = _run_once(fn, world, extra)
    for r, v in res.items():
        assert not isinstance(v, str), v
    return res


def test_collectives():
    res = _run(_w_collectives)
    r0, r1 = res[0], res[1]
    assert [d["r"] for d in r0["gather_obj"]] == [0, 1]
    assert [d["t"] for d in r0["gather_obj"]] == [[0], [1]]
    assert r0["gather_t"] == [[0.0, 1.0], [0.0, 1.0, 2.0]] and r1["gather_t"] is None
    assert r0["reduce"] == 1.5      # (1+2)/2 on rank 0
    assert r1["bcast"] == {"x": 5}
    assert r0["mean"] == r1["mean"] == 0.5


def _w_ddp(rank, world, port, q):
    try:
        pdist = _init(rank, world, port)
        from pytorch_distributed_template_amd.parallel import wrap_ddp
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(6, 4), torch.nn.ReLU(), torch.nn.Linear(4, 3))
        ref = torch.nn.Sequential(torch.nn.Linear(6, 4), torch.nn.ReLU(), torch.nn.Linear(4, 3))
        ref.load_state_dict(model.state_dict())
        ddp = wrap_ddp(model, torch.device("cpu"), bucket_cap_mb=1)
        torch.manual_seed(1)
        X = torch.randn(8, 6)
        Y = torch.randint(0, 3, (8,))
        xs, ys = X[rank * 4:(rank + 1) * 4], Y[rank * 4:(rank + 1) * 4]
        torch.nn.functional.cross_entropy(ddp(xs), ys).backward()
        torch.nn.functional.cross_entropy(ref(X), Y).backward()
        diffs = [float((a.grad - b.grad).abs().max()) for a, b in zip(model.parameters(), ref.parameters())]
        q.put((rank, {"diff": max(diffs)}))
        pdist.cleanup()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_ddp_gradients_equal_single_process():
    res = _run(_w_ddp)
    assert res[0]["diff"] < 1e-6 and res[1]["diff"] < 1e-6


def _w_sampler(rank, world, port, q):
    try:
        pdist = _init(rank, world, port)
        from pytorch_distributed_template_amd.data import MnistDataLoader
        tl = MnistDataLoader("/nonexistent", batch_size=16, shuffle=True, num_workers=0, training=True,
                             synthetic_size=64)
        tl.set_epoch(0)
        e0 = list(iter(tl.sampler))
        tl.set_epoch(1)
        e1 = list(iter(tl.sampler))
        vl = MnistDataLoader("/nonexistent", batch_size=16, shuffle=False, num_workers=0, training=False,
                             synthetic_size=37)
        q.put((rank, {"e0": e0, "e1": e1, "val": list(iter(vl.sampler))}))
        pdist.cleanup()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_sampler_sharding_set_epoch_and_unpadded_eval():
    res = _run(_w_sampler)
    assert res[0]["e0"] != res[0]["e1"]                      # Q6: reshuffle per epoch
    assert set(res[0]["e0"]).isdisjoint(res[1]["e0"])
    v = res[0]["val"] + res[1]["val"]
    assert sorted(v) == list(range(37))                      # Q9: no duplicates / padding


def _w_config(rank, world, port, q, tmp):
    try:
        pdist = _init(rank, world, port)
        from pytorch_distributed_template_amd.config import ConfigParser
        cfg = {"name": "D", "trainer": {"save_dir": tmp, "verbosity": 2}}
        c = ConfigParser(cfg)
        pdist.synchronize()
        q.put((rank, {"dir": str(c.save_dir)}))
        pdist.cleanup()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_single_run_dir_across_ranks(tmp_path):
    res = _run(_w_config, 2, str(tmp_path))
    assert res[0]["dir"] == res[1]["dir"]
    runs = list((tmp_path / "D" / "train").iterdir())
    assert len(runs) == 1 and (runs[0] / "config.json").exists()


def _w_pretune(rank, world, port, q):
    try:
        _init(rank, world, port)
        from pytorch_distributed_template_amd.ops import native_ops as no
        calls = []

        def step():  # stands in for the tuning forward+backward: only rank 0 may run it
            calls.append(rank)
            assert no._tune_allowed()
            no._tuned()["nt5:test"] = 7

        no._tuned().pop("nt5:test", None)
        assert not no._tune_allowed()  # WORLD_SIZE > 1: ranks never time variants on their own
        no.pretune_distributed(step)
        q.put((rank, {"calls": calls, "entry": no._tuned().get("nt5:test"), "allowed": no._tune_allowed()}))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_pretune_broadcasts_rank0_table():
    res = _run(_w_pretune)
    assert res[0]["calls"] == [0] and res[1]["calls"] == []
    assert res[0]["entry"] == 7 and res[1]["entry"] == 7
    assert not res[0]["allowed"] and not res[1]["allowed"]


def _w_graph_preflight(rank, world, port, q):
    try:
        _init(rank, world, port)
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        # no capturable RCCL group on these CPU ranks: the check must fail on every rank and
        # every rank must learn it (the agreement all-reduce runs on the job's own group)
        ok, why = bench.graph_collectives_ok(torch.device("cpu"), world)
        q.put((rank, {"ok": ok, "why": why}))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_bench_graph_preflight_falls_back_on_every_rank():
    res = _run(_w_graph_preflight)
    assert res[0]["ok"] is False and res[1]["ok"] is False
    assert res[0]["why"] and res[1]["why"]

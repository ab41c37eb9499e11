#!/usr/bin/env python
"""Flagship training-step benchmark: ResNet-50, bf16, synthetic 3x224x224, DDP.

Metric (BASELINE.json): images/sec for the whole job (all ranks), ResNet-50
on synthetic 3x224x224 data with random-init weights, one process per GPU over
RCCL (xGMI) when N > 1. Weak scaling: the per-GPU batch is fixed.

Each timed step is a full training step: forward, softmax-cross-entropy,
backward (DDP bucketed all-reduce over RCCL overlapped with it), optimizer
step (SGD momentum + weight decay). Nothing is skipped or cached. N = 1 runs
the same path: a 1-rank RCCL process group and the DDP reducer (``--no-ddp``
drops both for an A/B). ``--graph`` captures the whole step -- kernels, DDP
reducer and its RCCL all-reduces -- once as a HIP graph and replays it (PyTorch's
whole-network DDP capture recipe, on the stream DDP was built on; at N > 1 a capture
+ replay of one RCCL all-reduce is checked first and the run falls back to eager
launches if it fails anywhere).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                    [--model resnet50|resnet152|vit_b_16] [--backend native|torch]

N > 1: either launch it under ``torch.distributed.run`` (one rank per GPU,
``--gpus`` must equal WORLD_SIZE), or run ``python bench.py --gpus N`` directly:
the parent (which never touches the GPU) checks that N GPUs are visible, starts
the N ranks through ``torch.distributed.run`` on 127.0.0.1 and exits with their
status; rank 0 prints the one JSON line. ``--device cpu`` rehearses the same
path on CPU ranks over gloo (plumbing tests; not a performance number).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_METRIC = "images/sec (whole node) ResNet-50 synthetic 3x224x224 at 1/2/4/8 MI355X"
# Reference-equivalent stack (stock PyTorch-ROCm: autocast bf16, channels_last,
# MIOpen convs/BN, torch optimizers, torch.nn.parallel.DistributedDataParallel over a
# 1-rank RCCL group -- the reference's wrapper, train.py:45-52) measured on one MI355X with
# this same harness (`bench.py --backend torch --batch B`, 20 timed steps), keyed by (model,
# per-GPU batch), see BASELINE.md. Scaled by N for N GPUs (weak scaling). The bs 2048 points
# need MIOpen's find db (profiles/miopen_db_bs2048, scripts/gpu_job.sh benchlong): a cold
# find at that batch runs ~20 min, and immediate mode without it falls back to naive kernels.
# Round 5 (profiles/bench_runs_round5.jsonl, r5e / r5f): resnet50 2048, resnet152 2048, vit_b_16
# 1024; round 6 (profiles/bench_runs_round6.jsonl, q01): resnet152 3072 (258.7 GiB), 20 timed
# steps; the bs 256 / 512 points are round 2-3 measurements.
STOCK_1GPU_IMG_S = {("resnet50", 256): 6605.4, ("resnet50", 512): 6863.8, ("resnet50", 2048): 6936.44,
                    ("resnet152", 2048): 2852.86, ("resnet152", 3072): 2838.07,
                    ("vit_b_16", 256): 3547.25, ("vit_b_16", 1024): 4089.11}
# The stock stack's BEST measured per-GPU throughput (and its batch): reported as
# ``vs_best_stock``, never as ``vs_baseline``.
STOCK_BEST_1GPU_IMG_S = {"resnet50": (6936.44, 2048), "resnet152": (2852.86, 2048), "vit_b_16": (4089.11, 1024)}
# Per-GPU batch: 2048 images (82 GiB of the 288 GiB HBM3E; weak scaling, so the
# 8-GPU job holds 16384 images). The stage-3/4 GEMMs (M = N*14*14, N*7*7) fill all
# 256 CUs only from ~512 images up and every per-launch cost amortises over more
# images; measured on one MI355X: 11.96k img/s at 512, 12.45k at 768, 12.66k at
# 1024, 13.01k at 1536, 13.09-13.11k at 2048 (profiles/bench_runs_round2.jsonl).
# ViT-B/16: 1024 images per GPU (52 GiB fp8 / 60 GiB bf16); measured on one MI355X,
# fp8: 6.46k img/s at 256, 6.96k at 512, 7.31k at 1024, 7.49k at 2048; bf16 5.38k at
# 1024 (stock autocast: 3.55k at 256, 4.06k at 1024). At 256 the host-side issue
# time (~35 ms) is close to the 40 ms step: the GPU idles between kernels.
# ResNet-152 (BASELINE config 4, "per-GPU batch sized to 288 GB HBM"): 3072 images, 255.8 GiB of
# the 268 GiB: 6.17k img/s (2560: 6.11k, 213 GiB; profiles/bench_runs_round5.jsonl r5l, r5f). The
# stem and stage-1 tensors then hold 2.47e9 elements -- past 2^31: the conv path's offsets are
# 64-bit or unsigned 32-bit (README "Performance")
DEFAULT_BATCH = {"resnet50": 2048, "resnet152": 3072, "vit_b_16": 1024}
# --graph: batches run eagerly and replayed (lr 0) before the timed run; losses must agree
GRAPH_CHECK_STEPS = 3
# --graph: relative difference allowed between the weight updates of one eager step and one
# replay from the same state (atomics in the split-K reductions reorder fp32 sums; a doubled
# or dropped gradient is a difference of ~0.5-1)
GRAPH_UPDATE_TOL = 2e-2


def _train_state(model, opt):
    """Every tensor a training step mutates: parameters, buffers (BN running statistics),
    the fp8 delayed-scaling states of the native ViT layers, optimizer state (momentum /
    Adam moments), the fused optimizer's bf16 weight shadows and device [lr, t] scalars."""
    ts = [p.detach() for p in model.parameters()] + list(model.buffers())
    for m in model.modules():
        for a in ("_pdt_fp8_meta", "_pdt_fp8_gmeta"):
            if isinstance(getattr(m, a, None), torch.Tensor):
                ts.append(getattr(m, a))
    for st in opt.state.values():
        ts += [v for v in st.values() if isinstance(v, torch.Tensor)]
    ts += [v for v in getattr(opt, "_shadows", {}).values() if isinstance(v, torch.Tensor)]
    ts += [v for v in getattr(opt, "_dev", {}).values() if isinstance(v, torch.Tensor)]
    seen, out = set(), []
    for t in ts:
        if t.data_ptr() not in seen:
            seen.add(t.data_ptr())
            out.append(t)
    return out


class _UpdateCheck:
    """The --graph preflight at the REAL lr: one eager step (before the capture, so the eager
    activations are released before the graph's private pool is reserved) and one replay,
    each from the same saved state on the same batch; ``rel`` = ||dW_eager - dW_replay|| /
    ||dW_eager|| over all parameters. Every mutated tensor is restored after each."""

    def __init__(self, model, opt, batch):
        self.opt = opt
        self.state = _train_state(model, opt)
        self.saved = [t.clone() for t in self.state]
        self.params = [p.detach() for p in model.parameters() if p.requires_grad]
        self.p0 = [p.clone() for p in self.params]
        self.batch = batch
        self.de = None

    @torch.no_grad()
    def restore(self):
        for t, s in zip(self.state, self.saved):
            t.copy_(s)
        if hasattr(self.opt, "sync_shadows"):
            # the bf16 weight shadows of the restored weights, registered under the new
            # parameter versions: else the capture below records a weight cast per layer that
            # every replay repeats, and a replay after a restore reads stale shadows
            self.opt.sync_shadows()

    def eager(self, side, gstep, sx, sy):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            sx.copy_(self.batch[0])
            sy.copy_(self.batch[1])
            gstep()
        torch.cuda.current_stream().wait_stream(side)
        with torch.no_grad():
            self.de = [p - q for p, q in zip(self.params, self.p0)]
        self.restore()
        torch.cuda.synchronize()

    @torch.no_grad()
    def replay(self, graph, sx, sy) -> float:
        self.restore()
        sx.copy_(self.batch[0])
        sy.copy_(self.batch[1])
        graph.replay()
        num = sum(float((p - q - d).double().pow(2).sum()) for p, q, d in zip(self.params, self.p0, self.de))
        den = sum(float(d.double().pow(2).sum()) for d in self.de)
        self.restore()
        torch.cuda.synchronize()
        return math.sqrt(num / den) if den > 0 else float("inf")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: 2048 for resnet50, 1024 for vit_b_16, else 256)")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--fp8", action="store_true", help="ViT: fp8 (e4m3/e5m2) GEMMs on the native path")
    ap.add_argument("--backend", default="native", choices=["native", "torch"])
    ap.add_argument("--lr", type=float, default=None, help="learning rate (default: 0.1 SGD / 1e-3 AdamW)")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--comm-hook", default=None, choices=[None, "bf16"])
    ap.add_argument("--graph", dest="graph", action="store_true", default=None,
                    help="capture the whole training step (DDP all-reduce included) in one HIP graph and "
                         "replay it")
    ap.add_argument("--eager", dest="graph", action="store_false",
                    help="launch the step's kernels one by one (the default)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--miopen-find", type=int, default=1, choices=[0, 1],
                    help="torch backend: 1 = cudnn.benchmark (MIOpen find), 0 = immediate mode")
    ap.add_argument("--dist-backend", default=None, choices=[None, "nccl", "gloo"],
                    help="gloo: rehearse N ranks sharing GPU 0 (gradient all-reduce on the host); default RCCL")
    ap.add_argument("--data", default="sampler", choices=["sampler", "pool"],
                    help="sampler: SyntheticImageNet index batches from DistributedSampler, images made on device "
                         "every step (the config loader); pool: two pre-made resident batches")
    ap.add_argument("--no-ddp", action="store_true",
                    help="N=1 only: no process group and no DDP wrapper (A/B against the default 1-rank "
                         "RCCL group + DDP reducer that every N>1 rank also runs)")
    ap.add_argument("--ddp-impl", default=None, choices=[None, "native", "torch"],
                    help="data-parallel wrapper: native = the framework's BucketedDDP reducer (default, the CPU "
                         "rehearsal too), torch = torch.nn.parallel.DistributedDataParallel (default for the stock "
                         "--backend torch on the GPU, the reference's stack)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo ranks on the host with stock torch ops (launcher/plumbing rehearsal)")
    ap.add_argument("--image-size", type=int, default=224, help="only for --device cpu rehearsals")
    a = ap.parse_args()
    if a.batch is None:
        a.batch = DEFAULT_BATCH.get(a.model, 256)
    if a.graph is None:
        # eager by default: once captured on the stream DDP was built on (see below) the
        # replayed step runs at the eager rate (ResNet-50 bs2048 14.06k vs 14.08k, bs512
        # 12.23k vs 12.27k; profiles/bench_runs_round3.jsonl s4z), and an N > 1 capture of
        # RCCL collectives is one more thing that can fail on the driver's node
        a.graph = False
    if a.graph and (a.backend != "native" or a.device != "cuda" or a.dist_backend == "gloo"):
        ap.error("--graph needs the native backend on the GPU with RCCL collectives")
    if a.device == "cpu":
        a.backend, a.dist_backend, a.graph = "torch", "gloo", False
    if a.ddp_impl is None:
        # the CPU rehearsal runs stock ops but the framework's reducer (what every GPU rank of
        # the native stack runs); only the stock GPU baseline uses torch's DDP
        a.ddp_impl = "torch" if (a.backend == "torch" and a.device == "cuda") or a.comm_hook else "native"
    elif a.image_size != 224:
        ap.error("--image-size is a CPU-rehearsal knob; GPU runs measure 224x224")
    return a


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int | None:
    """Self-launch for ``--gpus N`` without a launcher; None = run in-process.

    Runs before anything touches the GPU (``torch.cuda.device_count`` does not
    initialise HIP on this image): the ranks are children, never an exec."""
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    if args.device == "cuda" and args.dist_backend != "gloo":
        n = torch.cuda.device_count()
        if n < args.gpus:
            print(f"bench.py: --gpus {args.gpus} requested but only {n} GPU(s) are visible; refusing to report "
                  f"a {n}-GPU number as {args.gpus}", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def graph_collectives_ok(device, world, check_single=False):
    """Can this job's RCCL collectives be captured in a HIP graph and replayed? Checked before
    the training step is captured, on a throwaway process group (a failed capture cannot leave
    the main group's communicator in a bad state): warm one all-reduce eagerly, capture it on a
    side stream, replay, check the sum. World 1 needs no check (the N = 1 step capture itself
    exercises that path).

    The ranks agree TWICE on the main group: first on "every rank captured" -- only then does
    any rank replay (a replay joined by fewer ranks than the group would block forever, and
    ``--graph`` runs without the RCCL watchdog's async abort) -- and then on "every replay
    summed correctly". Returns (ok, reason)."""
    if world == 1 and not check_single:
        return True, None
    import torch.distributed as dist

    def agree(v):
        flag = torch.tensor([int(v)], dtype=torch.int32, device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())

    why, g, t, pg = None, None, None, None
    try:
        pg = dist.new_group(backend="nccl")
        t = torch.ones(4096, device=device)
        dist.all_reduce(t, group=pg)
        torch.cuda.synchronize()
        from pytorch_distributed_template_amd.utils import dist as pdist
        pdist.quiesce_for_capture(device)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            t.fill_(1.0)
            with torch.cuda.graph(g, stream=side):
                dist.all_reduce(t, group=pg)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 -- any failure means: run eager
        why, g = f"capture: {type(e).__name__}: {e}", None
    if not agree(g is not None):
        return False, why or "another rank could not capture its collectives"
    try:
        t.fill_(1.0)
        g.replay()
        torch.cuda.synchronize()
        if not bool((t == float(world)).all()):
            why = f"replayed all-reduce returned {t[0].item()} instead of {world}"
    except Exception as e:  # noqa: BLE001
        why = f"replay: {type(e).__name__}: {e}"
    if not agree(why is None):
        return False, why or "another rank's replayed all-reduce failed"
    return True, None


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return None


def _dtype_label(args) -> str:
    if args.backend == "torch":
        return "bf16 (autocast)" if args.device == "cuda" else "fp32 (cpu rehearsal)"
    if not args.fp8:
        return "bf16"
    from pytorch_distributed_template_amd.ops.native_ops import fp8_settings
    c = fp8_settings()
    return (f"fp8(e4m3 fwd GEMMs, {c['scaling']} scaling; {'e5m2' if c['dgrad'] else 'bf16'} dgrad GEMMs; "
            f"{'fp8' if c['attn'] else 'bf16'} attention; {'e5m2 x e4m3' if c['dgrad'] and c['wgrad'] else 'bf16'} "
            f"wgrad GEMMs)+bf16")


def pdist_ready() -> bool:
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def allreduce_probe(model, device, world, iters=10):
    """Time an all-reduce of one gradient-sized fp32 buffer on the job's process group
    (outside the timed region): the xGMI/RCCL evidence of a multi-GPU run, recorded in
    the JSON next to the throughput. busbw = 2(n-1)/n * bytes / time (ring-equivalent).
    None at N = 1: a 1-rank RCCL all-reduce moves no bytes between GPUs (it is a local
    copy), so its time says nothing about xGMI."""
    if not pdist_ready() or device.type != "cuda" or world == 1:
        return None
    n = sum(p.numel() for p in model.parameters() if p.requires_grad)
    buf = torch.ones(n, dtype=torch.float32, device=device)
    for _ in range(3):
        torch.distributed.all_reduce(buf)
    torch.cuda.synchronize()
    t = torch.empty(iters, dtype=torch.float64)
    for i in range(iters):
        t0 = time.perf_counter()
        torch.distributed.all_reduce(buf)
        torch.cuda.synchronize()
        t[i] = time.perf_counter() - t0
    ms = float(t.median()) * 1e3
    nbytes = n * 4
    return {"bytes": nbytes, "median_ms": round(ms, 3),
            "busbw_GBps": round(2 * (world - 1) / world * nbytes / (ms / 1e3) / 1e9, 1)}


@torch.no_grad()
def rank_consistency(model, device, world):
    """Do all ranks hold the same weights after the timed steps? Every rank applies the same
    averaged gradient with the same optimizer, so the parameters must be bitwise equal: per
    parameter an fp64 sum and sum of squares, all-reduced MAX and MIN over the ranks; any
    difference is rank divergence (a bucket reduced on some ranks only, a slot mix-up, a
    rank-local update). Reported in the JSON (``ranks_in_sync``), not hidden."""
    ps = [p.detach() for p in model.parameters()]
    v = torch.stack([p.double().sum() for p in ps] + [p.double().square().sum() for p in ps])
    hi, lo = v.clone(), v.clone()
    if pdist_ready() and world > 1:
        torch.distributed.all_reduce(hi, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(lo, op=torch.distributed.ReduceOp.MIN)
    diff = float((hi - lo).abs().max())
    return {"ranks_in_sync": diff == 0.0, "param_checksum": float(v[:len(ps)].sum()),
            "param_checksum_max_rank_diff": diff, "ranks_checked": world}


def any_rank(flag: bool, device) -> bool:
    """True on every rank if ``flag`` is True on any rank (so all ranks take the same exit)."""
    if not pdist_ready():
        return bool(flag)
    t = torch.tensor([int(bool(flag))], dtype=torch.int32, device=device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return bool(t.item())


def refuse(rank, rec, reason, json_out=None):
    """Print the record with ``value: null`` and the reason, and exit non-zero: a step that
    produced a non-finite loss, or a replayed graph that disagrees with the eager step, is
    not a throughput measurement."""
    rec = dict(rec, value=None, vs_baseline=None, error=reason)
    if rank == 0:
        line = json.dumps(rec)
        print(line, flush=True)
        if json_out:
            with open(json_out, "w") as f:
                f.write(line + "\n")
    print(f"bench.py: {reason}", file=sys.stderr, flush=True)
    sys.exit(3)


def heartbeat(rank, state, every_s=30.0):
    """Rank 0 prints a progress line to stderr every ``every_s`` seconds (first-step
    autotuning / MIOpen searches can run for minutes without other output)."""
    import threading
    stop = threading.Event()
    if rank != 0:
        return stop
    t0 = time.time()

    def run():
        while not stop.wait(every_s):
            print(f"[bench] {time.time() - t0:.0f}s phase={state['phase']} step={state['step']}", file=sys.stderr,
                  flush=True)

    threading.Thread(target=run, daemon=True).start()
    return stop


def main():
    args = parse()
    if args.graph:
        # DDP inside a captured graph: the RCCL watchdog must not query the captured work
        # (PyTorch's whole-network-capture recipe), set before the process group exists
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    from pytorch_distributed_template_amd.utils import dist as pdist
    from pytorch_distributed_template_amd.ops import fused
    from pytorch_distributed_template_amd import models
    from pytorch_distributed_template_amd.parallel import is_data_parallel, pretune_for_ddp, wrap_ddp
    from pytorch_distributed_template_amd.data.synthetic import SyntheticImageLoader, SyntheticImageNetLoader

    cpu = args.device == "cpu"
    shared = args.dist_backend == "gloo" and not cpu
    # N = 1 runs the same DDP-over-RCCL path as every rank of an N > 1 job: a 1-rank
    # process group (RCCL on the GPU) and the DDP reducer with its bucketed all-reduce
    one_rank_pg = args.gpus == 1 and not args.no_ddp
    device = pdist.init_distributed(backend=args.dist_backend, device_index=0 if shared else None,
                                    single_rank_group=one_rank_pg) if not cpu \
        else pdist.init_distributed(backend="gloo", single_rank_group=one_rank_pg)
    world = pdist.get_world_size()
    rank = pdist.get_rank()
    if cpu:
        device = torch.device("cpu")
    elif device.type != "cuda":
        raise SystemExit("bench.py needs a GPU (use --device cpu for a plumbing rehearsal)")
    state = {"phase": "setup", "step": 0}
    hb = heartbeat(rank, state)
    fused.set_backend(args.backend)
    torch.backends.cudnn.benchmark = bool(args.miopen_find)

    torch.manual_seed(1234)
    ctor = {"resnet50": models.resnet50, "resnet152": models.resnet152, "vit_b_16": models.vit_b_16}[args.model]
    kw = {"fp8": True} if args.fp8 else {}
    model = ctor(num_classes=1000, **kw).to(device).to(memory_format=torch.channels_last)
    from pytorch_distributed_template_amd.optim import FusedAdamW, FusedSGD
    if args.model.startswith("vit"):
        lr = 1e-3 if args.lr is None else args.lr
        opt_name = f"AdamW(lr={lr:g}, wd=0.05)"
        # capturable under --graph: lr and Adam's step count in device memory, so every replay
        # applies the bias corrections of its own step (optim/fused.py)
        opt = FusedAdamW(model.parameters(), lr=lr, weight_decay=0.05, capturable=args.graph) \
            if args.backend == "native" else torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=0.05)
    else:
        lr = 0.1 if args.lr is None else args.lr
        opt_name = f"SGD(lr={lr:g}, momentum=0.9, wd=5e-5)"
        opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5, capturable=args.graph) \
            if args.backend == "native" else torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9,
                                                             weight_decay=5e-5)
    dtype = "float32" if cpu else "bfloat16"
    if args.data == "pool":
        loader = SyntheticImageLoader(args.batch, num_samples=args.batch * (args.steps + args.warmup + 2) * world,
                                      dtype=dtype, pool=2, device=device, image_size=args.image_size)
        pooled = list(iter(loader))[:2]

        def next_batch(i):
            return pooled[i % 2]
    else:
        # the reference's data path: DistributedSampler shards the (synthetic) dataset over
        # the ranks; each step's index batch becomes images in one device launch
        loader = SyntheticImageNetLoader(args.batch, num_samples=args.batch * 64 * world, dtype=dtype,
                                         device=device, image_size=args.image_size)

        def _forever():
            epoch = 0
            while True:
                loader.set_epoch(epoch)
                for b in loader:
                    if b[0].shape[0] == args.batch:
                        yield b
                epoch += 1

        _it = _forever()

        def next_batch(i):
            return next(_it)
    autocast = args.backend == "torch" and not cpu
    dev_type = device.type

    def _pretune_step():
        x, y = next_batch(0)
        fused.softmax_cross_entropy(model(x), y).backward()

    # N ranks: rank 0 tunes the kernel variants once and broadcasts them (no per-rank timing)
    pretune_for_ddp(model, _pretune_step)
    ar = allreduce_probe(model, device, world)
    graph_fallback = None
    graph_check, bad = None, False
    if args.graph and not args.no_ddp:
        ok, graph_fallback = graph_collectives_ok(device, world)
        if not ok:
            print(f"[bench] HIP-graph capture of the RCCL collectives failed ({graph_fallback}); running eager",
                  file=sys.stderr, flush=True)
            args.graph = False
    side = torch.cuda.Stream() if args.graph else None
    if side is not None:  # graph capture of DDP: the reducer is built on the capture side stream
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            model = wrap_ddp(model, device, bucket_cap_mb=args.bucket_mb, broadcast_buffers=False,
                             gradient_as_bucket_view=True, comm_hook=args.comm_hook, impl=args.ddp_impl)
    else:
        model = wrap_ddp(model, device, bucket_cap_mb=args.bucket_mb, broadcast_buffers=False,
                         gradient_as_bucket_view=True, comm_hook=args.comm_hook, impl=args.ddp_impl)

    def step(i):
        x, y = next_batch(i)
        opt.zero_grad(set_to_none=True)
        with torch.autocast(dev_type, dtype=torch.bfloat16, enabled=autocast):
            out = model(x)
            loss = fused.softmax_cross_entropy(out, y)
        loss.backward()
        opt.step()
        return loss

    if args.graph:
        # static input buffers; each replayed step first copies the next batch in
        x0, y0 = next_batch(0)
        sx, sy = x0.clone(), y0.clone()
        if getattr(x0, "pdt_nhwc_pad", None):  # keep the padded-NHWC view the stem reads in place
            from pytorch_distributed_template_amd.ops.native_ops import nhwc_padded_view
            cp = x0.pdt_nhwc_pad
            sbuf = nhwc_padded_view(x0, cp).clone(memory_format=torch.channels_last)
            sx = sbuf[:, :x0.shape[1]]
            sx.pdt_nhwc_pad = cp

        static_slots = bool(getattr(model, "static_grad_slots", False))

        def gstep():
            # fixed addresses for the capture: the reducer's bucket slots (gradients dropped,
            # the kernels write the slots), else gradients kept allocated and zeroed in place
            opt.zero_grad(set_to_none=static_slots)
            with torch.autocast(dev_type, dtype=torch.bfloat16, enabled=autocast):
                out = model(sx)
                loss = fused.softmax_cross_entropy(out, sy)
            loss.backward()
            opt.step()
            return loss

        # replay check: GRAPH_CHECK_STEPS batches run eagerly and then replayed, both at lr 0
        # (weights unchanged, so each loss depends only on its batch; BatchNorm normalises
        # with batch statistics in training mode): a capture that records the wrong stream,
        # buffer or order shows up as a loss mismatch instead of as throughput
        check_batches = [tuple(t.clone() for t in next_batch(i)) for i in range(GRAPH_CHECK_STEPS)]
        saved_lr = [g["lr"] for g in opt.param_groups]

        def set_lr(lrs):
            for g, lr in zip(opt.param_groups, lrs):
                g["lr"] = lr
            opt.refresh_scalars()

        side.wait_stream(torch.cuda.current_stream())
        eager_losses = []
        with torch.cuda.stream(side):
            # >= 11 eager iterations: DDP samples runtime stats (host-synchronising) on
            # iterations 1..10, which must all precede the capture
            for i in range(max(11, args.warmup)):
                xb, yb = next_batch(i)
                sx.copy_(xb)
                sy.copy_(yb)
                gstep()
            set_lr([0.0] * len(saved_lr))
            for xb, yb in check_batches:
                sx.copy_(xb)
                sy.copy_(yb)
                eager_losses.append(gstep().detach().clone())
        torch.cuda.current_stream().wait_stream(side)
        # the losses at lr 0 are blind to the gradient's SCALE (a doubled gradient gives the
        # same loss): one eager step here and one replay after the capture, from the same
        # state and batch at the real lr, must also move the weights by the same amount
        set_lr(saved_lr)
        upd = _UpdateCheck(model, opt, check_batches[0])
        upd.eager(side, gstep, sx, sy)
        set_lr([0.0] * len(saved_lr))
        # hand the warm-up's cached activation blocks back before the capture allocates the
        # graph's private pool: otherwise both stay reserved (2x the activations: ResNet-152
        # at 2048 images/GPU would not fit in 288 GB)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        pdist.quiesce_for_capture(device)  # the RCCL watchdog retires the warm-up's collectives first
        graph = torch.cuda.CUDAGraph()
        # captured on the stream DDP was built and warmed up on: DDP binds its gradient
        # accumulators to that stream (torch.cuda.graph's own private stream: NaN gradients)
        with torch.cuda.graph(graph, stream=side):
            static_loss = gstep()

        graph_losses = []
        for xb, yb in check_batches:
            sx.copy_(xb)
            sy.copy_(yb)
            graph.replay()
            graph_losses.append(static_loss.detach().clone())
        set_lr(saved_lr)
        step_rel = upd.replay(graph, sx, sy)
        del upd
        le = torch.stack(eager_losses).double().cpu()
        lg = torch.stack(graph_losses).double().cpu()
        rel = float(((le - lg).abs() / le.abs().clamp_min(1e-12)).max())
        graph_check = {"eager": [round(float(v), 6) for v in le], "replay": [round(float(v), 6) for v in lg],
                       "max_rel_diff": rel, "param_update_rel_diff": step_rel}
        del check_batches
        bad = not (torch.isfinite(le).all() and torch.isfinite(lg).all() and rel <= 1e-3 and
                   step_rel <= GRAPH_UPDATE_TOL)

        def step(i):  # noqa: F811
            xb, yb = next_batch(i)
            sx.copy_(xb)
            sy.copy_(yb)
            graph.replay()
            return static_loss

    # vs_baseline only against the stock stack measured at the SAME per-GPU batch (else
    # null); the ratio to the stock stack's best measured batch is a separately named field
    stock = STOCK_1GPU_IMG_S.get((args.model, args.batch))
    stock_ref = f"stock PyTorch-ROCm at per-GPU batch {args.batch}" if stock else None
    best = STOCK_BEST_1GPU_IMG_S.get(args.model)

    def record(value, ms, extra):
        cfg = {"model": args.model, "global_batch": args.batch * world, "per_gpu_batch": args.batch,
               "seq_len": None, "image_size": args.image_size, "parallelism": f"dp{world}",
               "backend": args.backend, "optimizer": opt_name,
               "bucket_cap_mb": args.bucket_mb,
               "dist_backend": (torch.distributed.get_backend() if pdist_ready() else "none (no process group)"),
               "ddp": is_data_parallel(model), "ddp_impl": type(model).__name__ if is_data_parallel(model) else None,
               "rccl_version": _rccl_version(), "device": args.device,
               "hip_graph": args.graph, "graph_fallback": graph_fallback, "graph_check": graph_check,
               "baseline": stock_ref,
               "vs_best_stock": ({"ratio": round(value / (best[0] * world), 4), "stock_img_s": best[0],
                                  "stock_per_gpu_batch": best[1]} if best and value else None),
               "grad_allreduce_probe": ar,
               # gradients a stock op produced outside the reducer's slots (each one a device copy)
               "ddp_fallback_copies": getattr(model, "fallback_copies", None),
               "ddp_fallback_shapes": sorted(getattr(model, "fallback_shapes", ()))[:16] or None,
               "max_mem_gib": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2) if not cpu else None}
        cfg.update(extra)
        return {
            "metric": BASELINE_METRIC if args.model == "resnet50" else f"images/sec (whole node) {args.model} synthetic",
            "value": round(value, 2) if value else None,
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3) if ms else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (stock * world), 4) if stock and value else None,
            "dtype": _dtype_label(args),
            "data": (f"synthetic 3x{args.image_size}x{args.image_size}, random-init weights; " +
                     ("SyntheticImageNet index batches from DistributedSampler, images generated on device each step"
                      if args.data == "sampler" else "two pre-made device-resident batches")),
            "config": cfg,
        }

    if args.graph and any_rank(bad, device):
        hb.set()
        refuse(rank, record(None, None, {}), f"the replayed graph disagrees with the eager step: {graph_check}",
               args.json_out)

    state["phase"] = "warmup"
    for i in range(args.warmup):
        state["step"] = i
        loss = step(i)
    sync = torch.cuda.synchronize if not cpu else (lambda: None)
    pdist.synchronize()
    sync()
    state["phase"] = "timed"
    t0 = time.perf_counter()
    cpu_issue = 0.0
    first_loss = None
    for i in range(args.steps):
        state["step"] = i
        c0 = time.perf_counter()
        loss = step(i)
        if i == 0:  # (a graph replay overwrites its static loss: keep a copy)
            first_loss = loss.detach().clone() if args.graph else loss
        cpu_issue += time.perf_counter() - c0
    pdist.synchronize()
    sync()
    elapsed = time.perf_counter() - t0
    hb.set()
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if pdist_ready():
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    loss_first = float(first_loss.item())
    loss_last = float(loss.item())
    ms = elapsed / args.steps * 1e3
    value = world * args.batch * args.steps / elapsed
    def _r(v):  # JSON has no NaN / inf: a non-finite loss is reported as null
        return round(v, 4) if math.isfinite(v) else None

    losses = {"loss_first": _r(loss_first), "loss_last": _r(loss_last), "final_loss": _r(loss_last)}
    # a broken step (NaN / inf loss on any rank) is not a throughput measurement
    if any_rank(not (math.isfinite(loss_first) and math.isfinite(loss_last)), device):
        refuse(rank, record(None, ms, losses), f"non-finite training loss (first {loss_first}, last {loss_last})",
               args.json_out)
    sync_rec = rank_consistency(model, device, world)
    if not sync_rec["ranks_in_sync"] and rank == 0:
        print(f"bench.py: WARNING ranks diverged after the timed steps: {sync_rec}", file=sys.stderr, flush=True)
    losses.update(sync_rec)
    # host enqueue cost of one step with an idle GPU (cpu_issue above includes the time the
    # host waits on a full submission queue while the GPU is busy)
    sync()
    h0 = time.perf_counter()
    step(args.steps)
    host_enqueue_ms = (time.perf_counter() - h0) * 1e3
    sync()

    losses.update({"cpu_issue_ms_per_step": round(cpu_issue / args.steps * 1e3, 3),
                   "host_enqueue_ms_idle_gpu": round(host_enqueue_ms, 3)})
    rec = record(value, ms, losses)
    if rank == 0:
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    pdist.cleanup()


if __name__ == "__main__":
    main()

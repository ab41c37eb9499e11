"""Per-op, per-shape device-time breakdown of the bench training step.

    python scripts/op_profile.py [--model resnet50] [--batch 2048] [--steps 2]

Runs bench.py's model/optimizer/data path (no DDP, one GPU) for a few warm-up steps,
then times every kernel-library launch of ``--steps`` steps with HIP events
(ops.native_ops.OpTimer) and prints the top entries: total ms per step, calls per
step, the entry point and its integer arguments (geometry, variant)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd import models  # noqa: E402
from pytorch_distributed_template_amd.data.synthetic import SyntheticImageLoader  # noqa: E402
from pytorch_distributed_template_amd.ops import fused, native_ops  # noqa: E402
from pytorch_distributed_template_amd.optim import FusedAdamW, FusedSGD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--top", type=int, default=70)
    ap.add_argument("--gap", type=int, default=40,
                    help="also print the N GEMM-family entries with the most time over their roofline floor")
    ap.add_argument("--cprofile", action="store_true",
                    help="instead: host-side cProfile of --steps steps (where the Python issue time goes)")
    ap.add_argument("--set", action="append", default=[], metavar="K=V",
                    help="environment switch for this run (e.g. PDT_FUSE_BN_AX=0), read at call time")
    a = ap.parse_args()
    for kv in a.set:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    os.environ["PDT_OP_TIMING"] = "0" if a.cprofile else "1"  # read at the library's first load
    fused.set_backend("native")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ctor = {"resnet50": models.resnet50, "resnet152": models.resnet152, "vit_b_16": models.vit_b_16}[a.model]
    model = ctor(num_classes=1000, **({"fp8": True} if a.fp8 else {})).to(dev).to(memory_format=torch.channels_last)
    if a.model.startswith("vit"):
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.05)
    else:
        opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    batches = list(iter(SyntheticImageLoader(a.batch, num_samples=2 * a.batch, pool=2, device=dev)))

    def step(i):
        x, y = batches[i % 2]
        opt.zero_grad(set_to_none=True)
        fused.softmax_cross_entropy(model(x), y).backward()
        opt.step()

    lib = native_ops._load()
    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    if a.cprofile:
        import cProfile
        import pstats
        import time
        pr = cProfile.Profile()
        # the autograd engine runs CUDA backward functions on its own device thread, which the
        # main thread's profiler does not see: every native backward enables a second
        # profiler on that thread for its own duration
        pb = cProfile.Profile()
        for cls in vars(native_ops).values():
            if isinstance(cls, type) and issubclass(cls, torch.autograd.Function) and "backward" in cls.__dict__:
                def wrapped(ctx, *g, _orig=cls.__dict__["backward"].__func__):
                    pb.enable()
                    try:
                        return _orig(ctx, *g)
                    finally:
                        pb.disable()
                cls.backward = staticmethod(wrapped)
        t0 = time.perf_counter()
        pr.enable()
        for i in range(a.steps):
            step(i)
        pr.disable()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host issue {1e3 * (t1 - t0) / a.steps:.1f} ms/step (under cProfile), drain {1e3 * (t2 - t1):.1f} ms")
        print("==== main thread (forward, optimizer)")
        pstats.Stats(pr).sort_stats("tottime").print_stats(40)
        print("==== autograd device thread (native backward functions)")
        pstats.Stats(pb).sort_stats("tottime").print_stats(40)
        return
    lib.records.clear()
    lib.enabled = True
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for i in range(a.steps):
        step(i)
    ev1.record()
    lib.enabled = False
    rows = lib.summary(top=10 ** 6)
    wall = ev0.elapsed_time(ev1) / a.steps
    total = sum(r[0] for r in rows) / a.steps
    print(f"{a.model} bs {a.batch}: {wall:.2f} ms/step wall, {total:.2f} ms/step inside library calls, "
          f"{sum(r[1] for r in rows) / a.steps:.0f} calls/step")
    by_name = {}
    for ms, n, name, key in rows:
        by_name[name] = by_name.get(name, 0.0) + ms / a.steps
    print("by entry point:")
    for name, ms in sorted(by_name.items(), key=lambda x: -x[1]):
        print(f"  {ms:8.3f} ms {100 * ms / total:5.1f}%  {name}")
    print("top (entry point, integer args):")
    for ms, n, name, key in rows[:a.top]:
        print(f"  {ms / a.steps:8.3f} ms {n // a.steps:3d}x  {name} {key}")
    if a.gap:
        gap_table(rows, a.steps, a.gap)


PEAK_FLOPS = 1.3e15  # achievable bf16 MFMA rate under load (gemm lab, 8192^3 at ~1.9 GHz)
PEAK_BYTES = 5.5e12  # achievable HBM bandwidth


def gemm_floor(name, k):
    """(GFLOP, GB, floor_us) of one call of a GEMM-family entry point from its integer args,
    or None. Bytes: the operands once and the output once (+ the fused epilogue's extra
    tensors), i.e. what an ideal kernel would move."""
    if name.startswith("pdt_conv_nt"):
        Hs, Ws, Cs, Nimg, Hm, Wm, Ncol, K = k[:8]
        M = Nimg * Hm * Wm
        fl = 2.0 * M * Ncol * K
        by = 2.0 * (Nimg * Hs * Ws * Cs + M * Ncol + Ncol * K)
        if name.startswith(("pdt_conv_nt_bnb", "pdt_conv_nt_ax")):
            by += 2.0 * M * Ncol  # y (BN-backward partials) / the second A operand or the written copy
        if name.endswith("bnb2"):
            by += 2.0 * M * Ncol
    elif name == "pdt_conv_wgrad" or name == "pdt_conv_wgrad_bn":
        M, Mo, No = k[:3]
        Hs, Ws, C, Hm, Wm = k[4:9]
        fl = 2.0 * M * Mo * No
        by = 2.0 * (M * Mo + (M // max(1, Hm * Wm)) * Hs * Ws * C) + 4.0 * Mo * No
    else:
        return None
    return fl / 1e9, by / 1e9, max(fl / PEAK_FLOPS, by / PEAK_BYTES) * 1e6


def gap_table(rows, steps, top):
    out, tot_t, tot_f = [], 0.0, 0.0
    for ms, n, name, key in rows:
        g = gemm_floor(name, key)
        if g is None:
            continue
        calls = n // steps
        t_us = 1e3 * ms / n
        tot_t += ms / steps
        tot_f += g[2] * calls / 1e3
        out.append(((t_us - g[2]) * calls / 1e3, calls, t_us, g, name, key))
    print(f"GEMM family: {tot_t:.2f} ms/step, floor {tot_f:.2f} ms (at {PEAK_FLOPS / 1e15:.2f} PF/s, "
          f"{PEAK_BYTES / 1e12:.1f} TB/s)")
    print("  excess_ms calls   us/call  floor_us  eff   GFLOP     GB  entry args")
    for ex, calls, t_us, (gf, gb, fl), name, key in sorted(out, key=lambda r: -r[0])[:top]:
        print(f"  {ex:8.3f} {calls:4d}  {t_us:8.1f}  {fl:8.1f} {100 * fl / t_us:4.0f}%  {gf:6.1f} {gb:6.2f}  {name} {key}")


if __name__ == "__main__":
    main()

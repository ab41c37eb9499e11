"""How close the fused BN-backward data-gradient GEMMs (pdt_conv_nt_bnb, csrc/conv_nt_tile.inc
BNB epilogue) run to the HBM roofline on the ResNet-50 bs-2048 1x1 shapes.

For each shape: the bytes the launch must move (dY, the BN input y, the addend and both ReLU
bit masks when present, the dA output, the partial rows), the time of the shipped tuned
variant and of every applicable variant, and a streaming reference from the same box
(``torch.add(y, addend, out=o)``: 2 reads + 1 write of the output size). Prints one line per
(shape, variant) with GB/s and the fraction of the streaming reference.

    python scripts/bnb_roofline.py [--batch 2048] [--variants 2,7,12,17,22,27,38-41] [--shapes 14:256:1024]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

# (H, K = dY channels, Ncol = dA channels, addend + addend mask, BN mask): the 1x1 data
# gradients that carry the BN-backward epilogue in a ResNet-50 step (conv1 of a block feeds
# the previous block's output unit: addend + both masks; conv3 feeds bn2: gate from y)
SHAPES = [(56, 64, 256, 1), (56, 128, 256, 1), (28, 128, 512, 1), (14, 256, 1024, 1), (7, 512, 2048, 1),
          (56, 256, 64, 0), (28, 512, 128, 0), (14, 1024, 256, 0), (7, 2048, 512, 0)]


def _ids(spec):
    out = []
    for part in spec.replace("+", ",").split(","):  # ('+' too: gpu_job.sh turns commas into spaces)
        lo, _, hi = part.partition("-")
        out += list(range(int(lo), int(hi or lo) + 1))
    return out


def timeit(fn, reps=5, rounds=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return statistics.median(ts) * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--variants", default="2,7,12,17,22,27,38-41")
    ap.add_argument("--shapes", default="", help="H:K:N[,H:K:N...] subset of SHAPES (e.g. for a counter pass)")
    ap.add_argument("--no-ref", action="store_true", help="skip the streaming reference (counter passes)")
    a = ap.parse_args()
    lib = no._load()
    table = no._tuned()
    torch.manual_seed(0)
    keep = {tuple(int(x) for x in t.split(":")) for t in a.shapes.split(",") if t}
    for H, K, N, boundary in SHAPES:
        if keep and (H, K, N) not in keep:
            continue
        M = a.batch * H * H
        dy = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
        wt = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
        y = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        addend = torch.randn(M, N, device="cuda").to(torch.bfloat16) if boundary else None
        amask = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device="cuda") if boundary else None
        bmask = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device="cuda") if boundary else None
        mean = torch.randn(N, device="cuda") * 0.1
        scale = torch.rand(N, device="cuda") + 0.5
        shift = torch.randn(N, device="cuda") * 0.1
        geo = (H, H, K, a.batch, H, H, N, K, K, 1, 1, 0, 0, -1, -1, 1, 1, H, H, 1, 1, 0, 0, N)
        key = f"ntb2:{H},{H},{K},{a.batch},{H},{H},{N},{K},1,1,1,1,1,{boundary},{boundary}"
        tuned = int(table.get(key, -1))
        ntm_max = max(lib.pdt_conv_nt_bnb_rows(M, N, K, v) for v in range(lib.pdt_conv_nt_num_variants()))
        part = torch.empty(2 * ntm_max * N + lib.pdt_rows_reduce_workspace(ntm_max, N), device="cuda")
        nbytes = M * K * 2 + M * N * 2 * (2 + int(boundary)) + (2 * M * N // 8 if boundary else 0)

        def run(v):
            R = lib.pdt_conv_nt_bnb_rows(M, N, K, v)
            return lib.pdt_conv_nt_bnb(no._p(dy), no._p(wt), no._p(out), no._p(addend), no._p(amask), *geo, int(v),
                                       no._p(y), no._p(mean), no._p(scale), no._p(shift), no._p(bmask), no._p(part),
                                       1, 0, R, no._s())

        o2 = torch.empty_like(out)
        ref_b = 3 * M * N * 2
        t_ref = 1.0 if a.no_ref else timeit(lambda: torch.add(y, out if addend is None else addend, out=o2))
        ref_bw = ref_b / t_ref
        print(f"H{H} K{K} N{N} {'boundary' if boundary else 'inner'}: M={M} bytes={nbytes / 1e9:.2f} GB  "
              f"stream ref {ref_bw / 1e12:.2f} TB/s  tuned v{tuned}", flush=True)
        cand = sorted(set(_ids(a.variants) + ([tuned] if tuned >= 0 else [])))
        for v in cand:
            rc = run(v)
            if rc == no.NOT_APPLICABLE:
                continue
            no._chk(rc, f"bnb v{v}")
            t = timeit(lambda: run(v))
            bw = nbytes / t
            print(f"   v{v:3d}{'*' if v == tuned else ' '} {t * 1e6:8.1f} us  {bw / 1e12:5.2f} TB/s  "
                  f"{bw / ref_bw * 100:5.1f}% of stream  floor {nbytes / ref_bw * 1e6:7.1f} us", flush=True)
        del dy, wt, y, out, addend, amask, bmask, part, o2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""A/B two conv_nt (bf16) or gemm_f8 variants on the ViT-B/16 linear shapes and a few
ResNet-50 bs2048 1x1 GEMM shapes: interleaved rounds, median time per variant.

    python scripts/ab_variant.py --bf16 36,37 --f8 10     (or 36/37: gpu_job.sh turns commas into spaces)
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

SHAPES = [(50432, 2304, 768), (50432, 768, 768), (50432, 3072, 768), (50432, 768, 3072), (50432, 768, 2304),
          (802816 * 2, 256, 64), (200704 * 2, 512, 128), (200704 * 2, 128, 512), (50176 * 2, 1024, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bf16", default="36,37")
    ap.add_argument("--f8", default="10")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    vb = [int(v) for v in a.bf16.replace("/", ",").split(",") if v.isdigit()]  # "/" also separates
    vf = [int(v) for v in a.f8.replace("/", ",").split(",") if v.isdigit()]
    lib = no._load()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        geo = dict(Hs=1, Ws=1, Cs=K, Nimg=M, Hm=1, Wm=1, Ncol=N, K=K, ldb=K, sh=1, sw=1, oh0=0, ow0=0, dh=1, dw=1,
                   nth=1, ntw=1, Ho=1, Wo=1, osh=1, osw=1, oph=0, opw=0, ldo=N)
        ref = None
        runs = {}
        for v in vb:
            runs[f"bf16 v{v}"] = (lambda v=v: lib.pdt_conv_nt(*no._nt_args(x, w, y, None, None, geo, 0, v)))
        if K % 128 == 0:
            x8, dx = no.quantize_fp8(x, no.E4M3)
            w8, dw = no.quantize_fp8(w, no.E4M3)
            y8 = torch.empty_like(y)
            for v in vf:
                runs[f"fp8 v{v}"] = (lambda v=v: no.gemm_f8(x8, w8, y8, dx, dw, variant=v))
        t = {k: [] for k in runs}
        outs = {}
        for k, fn in runs.items():
            fn()
            torch.cuda.synchronize()
            outs[k] = (y if k.startswith("bf16") else y8).clone()
        for _ in range(a.rounds):
            for k, fn in runs.items():
                e0.record()
                for _ in range(5):
                    fn()
                e1.record()
                e1.synchronize()
                t[k].append(e0.elapsed_time(e1) / 5)
        fl = 2.0 * M * N * K
        line = f"M={M} N={N} K={K}:"
        for k in runs:
            med = statistics.median(t[k])
            line += f"  {k} {med * 1e3:7.1f} us ({fl / med / 1e9:5.0f} TF)"
        # agreement between variants of the same dtype
        kb = [k for k in outs if k.startswith("bf16")]
        kf = [k for k in outs if k.startswith("fp8")]
        for ks in (kb, kf):
            for k in ks[1:]:
                d = (outs[k].float() - outs[ks[0]].float()).abs().max().item()
                line += f"  |{k}-{ks[0]}|max={d:.3g}"
        print(line, flush=True)


if __name__ == "__main__":
    main()

"""Time every weight-gradient variant (csrc/conv_wgrad.hip) on the ViT-B/16 bs256 linear
shapes and the ResNet-50 bs1024 conv shapes; prints per shape the best variant of the
first 28 (register-staged) and of any later ids, and TF/s.

Round-2 A/B (profiles/wgrad_lds_dma_ring_ab_round2.txt): an LDS-DMA (global_load_lds)
2-stage ring as ids 28..35 lost to the register-staged 1-stage 128x128 tile (3
workgroups per CU) on 13 of 16 shapes (0.5-0.9x) and tied on the rest; not kept.

    python scripts/wgrad_variants.py [--resnet-batch 1024]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def shapes(nb):
    out = []
    for Mo, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):  # ViT: dW[Mo][K], M = 256 * 197 tokens
        out.append((f"vit {Mo}x{K}", dict(M=50432, Mo=Mo, No=K, ldy=Mo, Hs=1, Ws=1, C=K, Hm=1, Wm=1, sh=1, sw=1,
                                          oh0=0, ow0=0, dh=1, dw=1, ntw=1), (50432, K)))
    for H, cin, mid, cout in ((56, 256, 64, 256), (28, 512, 128, 512), (14, 1024, 256, 1024), (7, 2048, 512, 2048)):
        M = nb * H * H
        out.append((f"r50 {H}x{H} 1x1 {cin}->{mid}", dict(M=M, Mo=mid, No=cin, ldy=mid, Hs=H, Ws=H, C=cin, Hm=H, Wm=H,
                                                           sh=1, sw=1, oh0=0, ow0=0, dh=1, dw=1, ntw=1), (nb * H * H, cin)))
        out.append((f"r50 {H}x{H} 3x3 {mid}", dict(M=M, Mo=mid, No=9 * mid, ldy=mid, Hs=H, Ws=H, C=mid, Hm=H, Wm=H,
                                                   sh=1, sw=1, oh0=-1, ow0=-1, dh=1, dw=1, ntw=3), (nb * H * H, mid)))
        out.append((f"r50 {H}x{H} 1x1 {mid}->{cout}", dict(M=M, Mo=cout, No=mid, ldy=cout, Hs=H, Ws=H, C=mid, Hm=H,
                                                           Wm=H, sh=1, sw=1, oh0=0, ow0=0, dh=1, dw=1, ntw=1),
                    (nb * H * H, mid)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--resnet-batch", type=int, default=1024)
    args = ap.parse_args()
    lib = no._load()
    nv = lib.pdt_wgrad_num_variants()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot_old = tot_new = 0.0
    for name, a, xshape in shapes(args.resnet_batch):
        dy = torch.randn(a["M"], a["Mo"], device="cuda").to(torch.bfloat16)
        x = torch.randn(*xshape, device="cuda").to(torch.bfloat16)
        out = torch.empty(a["Mo"] * a["No"], device="cuda")
        ref = None
        t = {}
        for v in range(nv):
            no.conv_wgrad(dy, x, out, variant=v, **a)
            if ref is None:
                ref = out.clone()
            else:
                e = ((out - ref).norm() / ref.norm()).item()
                assert e < 1e-3, (name, v, e)
            ev0.record()
            for _ in range(5):
                no.conv_wgrad(dy, x, out, variant=v, **a)
            ev1.record()
            ev1.synchronize()
            t[v] = ev0.elapsed_time(ev1) / 5
        fl = 2.0 * a["M"] * a["Mo"] * a["No"]
        bo = min(range(28), key=lambda v: t[v])
        if nv <= 28:
            print(f"{name:28s} v{bo:2d} {t[bo] * 1e3:8.1f} us ({fl / t[bo] / 1e9:5.0f} TF)", flush=True)
            tot_old += t[bo]
            tot_new += t[bo]
            continue
        bn = min(range(28, nv), key=lambda v: t[v])
        tot_old += t[bo]
        tot_new += min(t[bo], t[bn])
        print(f"{name:28s} old v{bo:2d} {t[bo] * 1e3:8.1f} us ({fl / t[bo] / 1e9:5.0f} TF) | "
              f"GL v{bn:2d} {t[bn] * 1e3:8.1f} us ({fl / t[bn] / 1e9:5.0f} TF)  x{t[bo] / t[bn]:.2f}  "
              f"all GL: " + " ".join(f"{v}:{t[v] * 1e3:.0f}" for v in range(28, nv)), flush=True)
    print(f"sum of best: old {tot_old:.3f} ms -> with GL {tot_new:.3f} ms")


if __name__ == "__main__":
    main()

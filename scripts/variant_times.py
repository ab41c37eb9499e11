"""Time every conv_nt variant (LDS-tiled 0..37 and streaming 38+) on the ResNet-50
1x1 GEMM shapes at batch 256 (argv[1]: another batch), forward (with BN statistics) and data-gradient
(plain) epilogues; prints the fastest few per shape with achieved HBM GB/s."""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

SHAPES = [  # K, N, H(out), stride  -- GEMM view: M = 256*H*H rows, K in, N out
    (64, 256, 56, 1), (64, 64, 56, 1), (256, 64, 56, 1), (256, 128, 56, 1), (128, 512, 28, 1),
    (512, 128, 28, 1), (256, 1024, 14, 1), (1024, 256, 14, 1), (128, 256, 56, 1), (256, 512, 28, 2),
]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    lib = no._load()
    nvar = lib.pdt_conv_nt_num_variants()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for K, N, H, s in SHAPES:
        Hi = H * s
        conv = nn.Conv2d(K, N, 1, s, 0, bias=False).cuda().to(memory_format=torch.channels_last)
        x = torch.randn(n, K, Hi, Hi, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        g = no._fwd_geom(n, Hi, Hi, K, conv)
        a = no._fwd_nt_geom(n, Hi, Hi, K, N, g)
        wb = no.bf16_weight(conv.weight)
        M = n * H * H
        y = torch.empty((n, N, H, H), dtype=torch.bfloat16, device="cuda", memory_format=torch.channels_last)
        for stats in (True, False):
            res = []
            for v in range(nvar):
                R = max(lib.pdt_conv_nt_stat_rows(M, N, K, v), 1)
                st = torch.empty(2 * R * N, device="cuda") if stats else None
                args = no._nt_args(x, wb, y, st, None, a, 0, v)
                rc = lib.pdt_conv_nt(*args)
                if rc == no.NOT_APPLICABLE:
                    continue
                assert rc == 0, (v, rc)
                best = float("inf")
                for _ in range(3):
                    ev0.record()
                    for _ in range(5):
                        lib.pdt_conv_nt(*args)
                    ev1.record()
                    ev1.synchronize()
                    best = min(best, ev0.elapsed_time(ev1) / 5 * 1e3)
                res.append((best, v))
            res.sort()
            bytes_ = (n * Hi * Hi * K + M * N) * 2
            top = " ".join(f"v{v}:{t:.1f}" for t, v in res[:5])
            stream = " ".join(f"v{v}:{t:.1f}" for t, v in res if v >= 38)
            print(f"n={n} K={K:4d} N={N:4d} H={H:2d} s={s} stats={int(stats)}  best {res[0][0]:6.1f}us "
                  f"{bytes_ / res[0][0] / 1e3:6.0f} GB/s | {top} | stream {stream}", flush=True)


if __name__ == "__main__":
    main()

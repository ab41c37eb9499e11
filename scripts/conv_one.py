"""Run one conv shape (fwd / dgrad / wgrad) a few times -- a target for
rocprofv3 counter collection, e.g.

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
        -d gpurun_out/pmc -o run --output-format csv -- python3 scripts/conv_one.py 64 56 256 1 1 fwd
"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def main():
    cin, h, cout, k, s = (int(v) for v in sys.argv[1:6])
    which = sys.argv[6] if len(sys.argv) > 6 else "fwd"
    n = int(os.environ.get("BATCH", "256"))
    iters = int(os.environ.get("ITERS", "5"))
    p = k // 2
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(n, cin, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = no._fwd_geom(n, h, h, cin, conv)
    wb = no.bf16_weight(conv.weight)
    y, _, _, _ = no._conv_forward(x, wb, n, h, h, cin, cout, g, with_stats=True)
    dy = torch.randn_like(y)
    dw = torch.empty((cout, cin, k, k), device="cuda", memory_format=torch.channels_last)
    w32 = conv.weight.detach().float()
    for _ in range(iters):
        if which == "fwd":
            no._conv_forward(x, wb, n, h, h, cin, cout, g, with_stats=True)
        elif which == "dgrad":
            no._conv_dgrad(dy, w32, n, h, h, cin, cout, g)
        else:
            no._conv_wgrad(dy, x, n, h, h, cin, cout, g, dw)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

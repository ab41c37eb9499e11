"""Patch embedding paths side by side on ViT-B/16 shapes: patchify + GEMM vs the channel-padded
implicit GEMM, errors vs an fp32 conv (tokens, weight and bias gradients).

    python scripts/probe_patch_embed.py
"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def err(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def main():
    for B in (4, 64):
        for mf in (torch.contiguous_format, torch.channels_last):
            torch.manual_seed(27)
            conv = nn.Conv2d(3, 768, 16, stride=16).cuda().to(memory_format=mf)
            x = torch.randn(B, 3, 224, 224, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            g = torch.randn(B, 196, 768, device="cuda")
            yr = conv(x.float()).flatten(2).transpose(1, 2)
            wr, br = torch.autograd.grad(yr, (conv.weight, conv.bias), g)
            for path in ("1", "0"):
                os.environ["PDT_PATCH_LINEAR"] = path
                conv.zero_grad(set_to_none=True)
                y = no.patch_embed(x, conv)
                y.backward(g.to(torch.bfloat16))
                print(f"B={B} {str(mf):24s} linear={path}: y {err(y, yr):.2e} dw {err(conv.weight.grad, wr):.2e} "
                      f"db {err(conv.bias.grad, br):.2e}", flush=True)


if __name__ == "__main__":
    main()

"""Fused attention fwd+bwd on the ViT-B/16 batch-256 shape, a few times -- a
target for rocprofv3 counter collection:

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
        -d gpurun_out/pmc_attn -o run --output-format csv -- python3 scripts/attn_one.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

B, T, H = int(os.environ.get("BATCH", "256")), 197, 12
qkv = torch.randn(B, T, 3 * H * 64, device="cuda").to(torch.bfloat16).requires_grad_(True)
g = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
for _ in range(int(os.environ.get("ITERS", "3"))):
    out = no.qkv_attention(qkv, H)
    out.backward(g)
torch.cuda.synchronize()
print("ok")

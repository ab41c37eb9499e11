"""fp8 attention forward + fused fp8 backward on the ViT-B/16 shape (B=1024 by default, T=197,
H=12), a few times -- a target for rocprofv3 counter passes (scripts/probes/attn_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

B, T, H = int(os.environ.get("BATCH", "1024")), 197, 12
torch.manual_seed(0)
qkv = (torch.randn(B, T, 3 * H * 64, device="cuda") * 1.5).to(torch.bfloat16).requires_grad_(True)
g = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
for _ in range(int(os.environ.get("ITERS", "3"))):
    out = no.qkv_attention(qkv, H, fp8=True)
    out.backward(g)
torch.cuda.synchronize()
print("ok")

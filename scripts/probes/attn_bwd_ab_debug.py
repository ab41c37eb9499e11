"""Debug: the fused fp8 attention backward of two library builds on the same inputs (the in-tree
build and PDT_AB_LIB), phase 1's fp32 dS (debug output) and d(qkv) compared element-wise."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

new = no._load()
old = ctypes.CDLL(os.environ.get("PDT_AB_LIB", "abtest/libpdt_old.so"))
B, T, H = 3, 197, 4
torch.manual_seed(B * 1000 + T)
qkv = (torch.randn(B, T, 3 * H * 64, device="cuda") * 1.5).to(torch.bfloat16)
dout = torch.randn(B, T, H * 64, device="cuda").to(torch.bfloat16)
out = torch.empty(B, T, H * 64, dtype=torch.bfloat16, device="cuda")
lse = torch.empty(B * H, T, dtype=torch.float32, device="cuda")
P = no._p
assert new.pdt_attn_fwd(P(qkv), P(out), P(lse), B, T, H, ctypes.c_float(0.125), no._s()) == 0
R = 64 * ((T + 63) // 64)
res = {}
for name, lib in (("new", new), ("old", old)):
    d8 = torch.full_like(qkv, float("nan"))
    dbg = torch.zeros(B * H, R, R, device="cuda")
    rc = lib.pdt_attn_bwd_f8_debug(ctypes.c_void_p(qkv.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                   ctypes.c_void_p(dout.data_ptr()), ctypes.c_void_p(lse.data_ptr()),
                                   ctypes.c_void_p(d8.data_ptr()), B, T, H, ctypes.c_float(0.125),
                                   ctypes.c_void_p(dbg.data_ptr()), ctypes.c_void_p(0))
    torch.cuda.synchronize()
    assert rc == 0, (name, rc)
    res[name] = (d8.float(), dbg)
(dn, sn), (do_, so) = res["new"], res["old"]
s_n, s_o = sn.view(B * H, R, R)[:, :T, :T], so.view(B * H, R, R)[:, :T, :T]
print("dS max|old|", s_o.abs().max().item(), "max|new|", s_n.abs().max().item(), "max|diff|", (s_n - s_o).abs().max().item())
diff = (s_n - s_o).abs() > 1e-3 * s_o.abs().max()
idx = diff.nonzero()
print("dS differing entries", idx.shape[0], "of", s_o.numel())
if idx.shape[0]:
    print(" first", idx[:8].tolist())
    print(" query rows hit", torch.unique(idx[:, 1])[:40].tolist())
    print(" key cols hit", torch.unique(idx[:, 2])[:40].tolist())
    r = idx[0]
    print(" sample new/old", s_n[r[0], r[1], :8].tolist(), s_o[r[0], r[1], :8].tolist())
for k, sl in (("dq", slice(0, H * 64)), ("dk", slice(H * 64, 2 * H * 64)), ("dv", slice(2 * H * 64, 3 * H * 64))):
    a, b = dn[..., sl], do_[..., sl]
    print(k, "rel err new vs old", ((a - b).norm() / b.norm()).item(), "finite", torch.isfinite(a).all().item())

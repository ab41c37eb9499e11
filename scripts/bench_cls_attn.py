"""Per-call time of the class-token attention kernels (csrc/attention_cls.hip) at the ViT-B/16
bench shape (B=1024, T=197, H=12), forward and backward, with HIP events."""
import ctypes
import json
import sys

import torch

B, T, H = 1024, 197, 12


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    lib = ctypes.CDLL(sys.argv[1])  # a .so holding pdt_cls_attn_fwd / _bwd (A/B: old vs new build)
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.pdt_cls_attn_fwd.argtypes = [P, P, P, I, I, I, P]
    lib.pdt_cls_attn_bwd.argtypes = [P, P, P, P, P, I, I, I, P]
    s = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    qkv = (torch.randn(B, T, 3 * H * 64, device="cuda") * 0.5).to(torch.bfloat16)
    o = torch.empty(B, H * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H, device="cuda", dtype=torch.float32)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    fwd = lambda: lib.pdt_cls_attn_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), B, T, H, s)
    bwd = lambda: lib.pdt_cls_attn_bwd(qkv.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                                       dqkv.data_ptr(), B, T, H, s)
    assert fwd() == 0 and bwd() == 0
    rec = {"fwd_us": round(timed(fwd), 1), "bwd_us": round(timed(bwd), 1),
           "checksum": float(dqkv.float().abs().sum()), "lib": sys.argv[1]}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()

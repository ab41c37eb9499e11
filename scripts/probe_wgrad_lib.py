"""ResNet-50 (batch 2048) 1x1 weight gradients dW = dY^T X: the native split-K kernel (every
variant, tuned) next to hipBLASLt through torch.mm(dY^T, X, out_dtype=float32) -- is the library
worth a tuner id for the plain (no BN-apply) ones?

    python scripts/probe_wgrad_lib.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

SHAPES = [(6422528, 64, 256), (6422528, 256, 64), (1605632, 128, 512), (1605632, 512, 128),
          (401408, 256, 1024), (401408, 1024, 256), (100352, 512, 2048), (100352, 2048, 512)]  # (P, Cout, Cin)


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    torch.manual_seed(0)
    lib = no._load()
    for P, Co, Ci in SHAPES:
        dy = torch.randn(P, Co, device="cuda").to(torch.bfloat16)
        x = torch.randn(P, Ci, device="cuda").to(torch.bfloat16)
        out = torch.empty(Co, Ci, device="cuda")
        a = dict(M=P, Mo=Co, No=Ci, ldy=Co, Hs=1, Ws=1, C=Ci, Hm=1, Wm=1, sh=1, sw=1, oh0=0, ow0=0, dh=1, dw=1, ntw=1)
        best = (1e9, -1)
        for v in [v for v in range(lib.pdt_wgrad_num_variants()) if v != lib.pdt_wgrad_halo_id()]:
            try:
                t = timeit(lambda: no.conv_wgrad(dy, x, out, variant=v, **a))
            except Exception:  # noqa: BLE001
                continue
            best = min(best, (t, v))
        no.conv_wgrad(dy, x, out, variant=best[1], **a)
        ref = out.clone()
        try:
            t_l = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
            got = torch.mm(dy.t(), x, out_dtype=torch.float32)
            err = ((got - ref).norm() / ref.norm()).item()
            lib_s = f"hipBLASLt {t_l:7.1f} us err {err:.1e}"
        except Exception as e:  # noqa: BLE001
            lib_s = f"hipBLASLt n/a ({type(e).__name__}: {str(e)[:80]})"
        fl = 2.0 * P * Co * Ci
        print(f"P={P} Cout={Co} Cin={Ci}: native {best[0]:7.1f} us (v{best[1]}, {fl / best[0] / 1e6:5.0f} TF) | {lib_s}",
              flush=True)
        del dy, x


if __name__ == "__main__":
    main()

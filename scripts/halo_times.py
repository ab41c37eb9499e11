"""Time the stride-1 3x3 convs of ResNet-50 at the bench batch (argv[1], default 2048):
every conv_nt variant (LDS-tiled, and the halo-patch kernels of csrc/conv3x3_halo.hip),
forward with the BatchNorm-statistics epilogue and data gradient with the fused
BatchNorm-backward epilogue; prints the best generic vs the best halo variant with
TFLOP/s (2 * M * Cout * 9 * Cin per call)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

SHAPES = [(64, 56), (128, 28), (256, 14), (512, 7)]  # C (= Cin = Cout), H = W


def timeit(fn, reps=3, inner=5):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(reps):
        ev0.record()
        for _ in range(inner):
            fn()
        ev1.record()
        ev1.synchronize()
        best = min(best, ev0.elapsed_time(ev1) / inner * 1e3)
    return best


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    lib = no._load()
    nvar = lib.pdt_conv_nt_num_variants()
    for C, H in SHAPES:
        torch.manual_seed(0)
        x = torch.randn(n, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, C, 3, 3, device="cuda") * 0.05).contiguous(memory_format=torch.channels_last)
        wb = no.bf16_weight(w)
        M = n * H * H
        flop = 2.0 * M * C * 9 * C
        g = dict(KH=3, KW=3, sh=1, sw=1, ph=1, pw=1, Ho=H, Wo=H)
        a = no._fwd_nt_geom(n, H, H, C, C, g)
        y = torch.empty_like(x)
        wt = torch.empty(C * 9 * C, dtype=torch.bfloat16, device="cuda")
        no._chk(lib.pdt_wt_dgrad(no._p(w), no._p(wt), C, 3, 3, C, 0, 0, 1, 3, 3, no._s()), "wt")
        ad = dict(a, oh0=1, ow0=1, dh=-1, dw=-1)
        mean = torch.zeros(C, device="cuda")
        sc = torch.ones(C, device="cuda")
        sh = torch.zeros(C, device="cuda")
        for kind in ("fwd+stats", "dgrad+bnb"):
            res = []
            for v in range(nvar):
                if kind == "fwd+stats":
                    R = max(lib.pdt_conv_nt_stat_rows(M, C, 9 * C, v), 1)
                    st = torch.empty(2 * R * C, device="cuda")
                    args = no._nt_args(x, wb, y, st, None, a, 0, v)
                    fn = lambda args=args: lib.pdt_conv_nt(*args)  # noqa: E731
                else:
                    R = max(lib.pdt_conv_nt_bnb_rows(M, C, 9 * C, v), 1)
                    part = torch.empty(2 * R * C, device="cuda")
                    fn = lambda v=v, part=part, R=R: lib.pdt_conv_nt_bnb(  # noqa: E731
                        no._p(x), no._p(wt), no._p(y), None, None, H, H, C, n, H, H, C, 9 * C, 9 * C, 1, 1, 1, 1, -1,
                        -1, 3, 3, H, H, 1, 1, 0, 0, C, v, no._p(x), no._p(mean), no._p(sc), no._p(sh), None,
                        no._p(part), 1, 0, R, no._s())
                rc = fn()
                if rc == no.NOT_APPLICABLE:
                    continue
                assert rc == 0, (kind, v, rc)
                res.append((timeit(fn), v))
            res.sort()
            gen = [r for r in res if lib.pdt_conv_nt_variant_kind(r[1]) != 2]
            halo = [r for r in res if lib.pdt_conv_nt_variant_kind(r[1]) == 2]
            line = f"n={n} C={C:3d} H={H:2d} {kind:10s}"
            if gen:
                line += f" | generic v{gen[0][1]:2d} {gen[0][0]:8.1f} us {flop / gen[0][0] / 1e6:6.0f} TF/s"
            if halo:
                line += " | halo " + " ".join(f"v{v}:{t:.1f}us/{flop / t / 1e6:.0f}TF" for t, v in halo)
            print(line, flush=True)
        # weight gradient: every wgrad variant (the last id is the halo kernel)
        wa = dict(M=M, Mo=C, No=9 * C, ldy=C, Hs=H, Ws=H, C=C, Hm=H, Wm=H, sh=1, sw=1, oh0=-1, ow0=-1, dh=1, dw=1,
                  ntw=3)
        dw = torch.empty((C, C, 3, 3), device="cuda").contiguous(memory_format=torch.channels_last)
        res = []
        for v in range(lib.pdt_wgrad_num_variants()):
            fn = lambda v=v: no._wgrad_launch(lib, x, x, dw, v, 1.0, False, wa)  # noqa: E731
            rc = fn()
            if rc == no.NOT_APPLICABLE:
                continue
            assert rc == 0, ("wgrad", v, rc)
            res.append((timeit(fn), v))
        res.sort()
        hv = lib.pdt_wgrad_halo_id()
        gen = [r for r in res if r[1] != hv]
        halo = [r for r in res if r[1] == hv]
        line = f"n={n} C={C:3d} H={H:2d} {'wgrad':10s} | generic v{gen[0][1]:2d} {gen[0][0]:8.1f} us " \
               f"{flop / gen[0][0] / 1e6:6.0f} TF/s"
        if halo:
            line += f" | halo {halo[0][0]:.1f}us/{flop / halo[0][0] / 1e6:.0f}TF"
        print(line, flush=True)
        del x, y


if __name__ == "__main__":
    main()

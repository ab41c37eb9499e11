"""Run every conv_nt tile variant on one geometry with fresh buffers and check
(a) the result against torch, (b) that the inputs were not modified (an
out-of-bounds store would show up here)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn as nn, torch.nn.functional as F
from pytorch_distributed_template_amd.ops import native_ops as no

shapes = [(2, 256, 56, 56, 512, 1, 2, 0), (2, 128, 56, 56, 128, 3, 2, 1), (4, 64, 56, 56, 64, 1, 1, 0),
          (4, 1024, 4, 4, 2048, 1, 2, 0), (4, 512, 2, 2, 512, 3, 1, 1), (4, 256, 8, 8, 256, 3, 1, 1)]
for (N, Cin, H, W, Cout, k, s, p) in shapes:
    torch.manual_seed(0)
    conv = nn.Conv2d(Cin, Cout, k, s, p, bias=False).cuda()
    x = torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = no._fwd_geom(N, H, W, Cin, conv)
    wb = no.bf16_weight(conv.weight)
    ref = F.conv2d(x.float(), conv.weight.detach().to(torch.bfloat16).float(), None, s, p)
    a = no._fwd_nt_geom(N, H, W, Cin, Cout, g)
    M = N * g["Ho"] * g["Wo"]
    for v in range(no._load().pdt_conv_nt_num_variants()):
        for with_stats in (False, True):
            xc, wc = x.clone(), wb.clone()
            guard = torch.full((1 << 20,), 7, dtype=torch.bfloat16, device="cuda")
            y = torch.empty_like(ref, dtype=torch.bfloat16, memory_format=torch.channels_last)
            R = no.conv_stat_rows(M, Cout, a["K"], v)
            st = torch.zeros(2 * R * Cout, device="cuda") if with_stats else None
            no.conv_nt(x, wb, y, stats=st, variant=v, **a)
            torch.cuda.synchronize()
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            ok_in = torch.equal(xc, x) and torch.equal(wc, wb) and bool((guard == 7).all())
            serr = 0.0
            if with_stats:
                ps = st.view(2, R, Cout).sum(1)
                serr = ((ps[0] - ref.sum((0, 2, 3))).abs().max() / ref.sum((0, 2, 3)).abs().max()).item()
            print(f"shape={(N, Cin, H, Cout, k, s)} v={v:2d} stats={int(with_stats)} err={err:.4f} "
                  f"stat_err={serr:.4f} inputs_ok={ok_in}", flush=True)

"""Numerics at the ACTUAL bench batch (2048 images / GPU), in the default GPU suite.

The large-M index paths (32-bit element offsets: the ResNet-50 stem activation is
2048 x 64 x 112 x 112 = 1.64 G elements, within 24 % of 2^31; BatchNorm partial-row
reductions over 25.7 M rows; split-K weight-gradient slabs) only occur at the
bench geometry. The fp32 references are computed with the convolutions chunked
along the batch (per-image ops, so chunking is exact) and BatchNorm over the FULL
batch, which keeps MIOpen on small, fast problems.

* the stem node (conv 7x7/2 + BN + ReLU + max-pool) and layer1.0 -> layer1.1 (bottleneck
  with downsample, then one whose conv1 applies layer1.0's BN in its A staging), forward and
  backward, vs fp32: relative Frobenius error no worse than max(3 x the stock bf16 autocast
  error, 0.03) (the yardstick of tests/test_bench_geometry_gpu.py); also at 2752 images,
  where the stem output and every 256-channel stage-1 tensor hold 2752 x 802 816 = 2.21e9
  elements -- past 2^31 (the unsigned 32-bit offsets of the A-staging BN apply and of the
  BN-backward epilogue, 64-bit everywhere else: ResNet-152 at 3072 images per GPU);
* 3 SGD steps of the whole ResNet-50 at bs 2048 on the native kernels vs the same
  steps in fp32 on the stock ops: the loss trajectory agrees to 1 %.
"""
import contextlib

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

from pytorch_distributed_template_amd.ops import fused  # noqa: E402
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402

BS = 2048


def nrmerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def setup_module(module):
    assert no.available(), "native library must be built and loaded on GPU runs"
    no.require()
    torch.backends.cudnn.benchmark = False


@contextlib.contextmanager
def chunked_fp32_convs(chunk=256):
    """nn.Conv2d.forward evaluated in batch chunks (exact: a conv is per image)."""
    orig = nn.Conv2d.forward

    def fwd(self, x):
        if x.shape[0] <= chunk:
            return orig(self, x)
        return torch.cat([orig(self, x[i:i + chunk]) for i in range(0, x.shape[0], chunk)])

    nn.Conv2d.forward = fwd
    try:
        yield
    finally:
        nn.Conv2d.forward = orig


def _grads(params):
    return [p.grad.detach().float().clone() for p in params]


def _compare(name, fn, x, params, tol=0.03, need_dx=True):
    # native (need_dx=False: the input takes no gradient -- the bench's stem path, which
    # reads the loader's padded-NHWC batch in place through the space-to-depth GEMM)
    for p in params:
        p.grad = None
    fused.set_backend("native")
    xn = x.detach().clone().requires_grad_(True) if need_dx else x
    yn = fn(xn)
    gy = _cl(torch.randn(yn.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(7))
             .to(torch.bfloat16))
    yn.backward(gy)
    out_n, gp_n = yn.detach().float(), _grads(params)
    dx_n = xn.grad.float() if need_dx else None
    del yn, xn
    def stock(autocast):
        for p in params:
            p.grad = None
        fused.set_backend("torch")
        xr = x.detach().float().requires_grad_(need_dx)
        with chunked_fp32_convs(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            yr = fn(xr)
        yr.float().backward(gy.float() if not autocast else gy.to(yr.dtype))
        fused.set_backend("auto")
        res = (yr.detach().float(), xr.grad.float() if need_dx else None, _grads(params))
        del yr, xr
        return res

    # fp32 reference (stock ops, chunked convs), then the stock bf16 autocast yardstick: the
    # gradient of a conv feeding a BatchNorm cancels strongly (BN's dy has zero mean and is
    # orthogonal to y per channel), so bf16 rounding alone costs it ~7-14 % (round 2 logs)
    yr, dxr, pr = stock(False)
    ya, dxa, pa = stock(True)
    pairs = [(out_n, yr, ya)] + ([(dx_n, dxr, dxa)] if need_dx else []) + list(zip(gp_n, pr, pa))
    en = [nrmerr(n_, r_) for n_, r_, _ in pairs]
    ea = [nrmerr(a_, r_) for _, r_, a_ in pairs]
    del yr, dxr, pr, ya, dxa, pa, pairs
    torch.cuda.empty_cache()
    msg = f"{name}: native {['%.4f' % e for e in en]} autocast {['%.4f' % e for e in ea]}"
    print(msg)
    assert all(e <= max(3 * a, tol) for e, a in zip(en, ea)), msg
    return out_n


def _batch(i, bs=BS):
    """The bench's batch: SyntheticImageNet samples, NHWC padded to 4 channels (pdt_nhwc_pad)."""
    from pytorch_distributed_template_amd.data.synthetic import SyntheticImageNet
    x, y = SyntheticImageNet(bs * 4, seed=5, device="cuda").collate(list(range(i * bs, (i + 1) * bs)))
    assert getattr(x, "pdt_nhwc_pad", None) == 4
    return x


@pytest.mark.timeout(900)
@pytest.mark.parametrize("bs", [BS, 2752])
def test_resnet50_stem_and_layer1_at_bench_batch_vs_fp32(bs):
    from pytorch_distributed_template_amd.models import resnet50
    torch.manual_seed(41)
    m = resnet50(num_classes=1000).cuda().to(memory_format=torch.channels_last)
    x = _batch(0, bs)
    if bs == BS:
        assert bs * 64 * 112 * 112 > 1.6e9  # the stem activation is within 24 % of 2^31 elements
    else:
        assert bs * 64 * 112 * 112 > 2 ** 31 and bs * 256 * 56 * 56 > 2 ** 31
    stem = _compare(f"stem bs{bs}", lambda t: fused.conv_bn_relu_maxpool(t, m.conv1, m.bn1), x,
                    [m.conv1.weight, m.bn1.weight, m.bn1.bias], need_dx=False)
    del x
    b0, b1 = m.layer1[0], m.layer1[1]
    _compare(f"layer1.0-1 bs{bs}", lambda t: fused.bottleneck_chain(t, [b0, b1]),
             _cl(stem.to(torch.bfloat16)),
             [b0.conv1.weight, b0.conv3.weight, b0.bn3.weight, b0.downsample[0].weight, b1.conv1.weight,
              b1.conv2.weight, b1.bn1.weight])


@pytest.mark.timeout(600)
def test_resnet50_three_step_loss_trajectory_bs2048_native_vs_fp32():
    from pytorch_distributed_template_amd.models import resnet50
    from pytorch_distributed_template_amd.optim import FusedSGD
    torch.manual_seed(42)
    m_n = resnet50(num_classes=1000).cuda().to(memory_format=torch.channels_last)
    m_r = resnet50(num_classes=1000).cuda().to(memory_format=torch.channels_last)
    m_r.load_state_dict(m_n.state_dict())
    xs = [_batch(i) for i in range(3)]
    ys = [torch.randint(0, 1000, (BS,), device="cuda", generator=torch.Generator("cuda").manual_seed(30 + i))
          for i in range(3)]
    o_n = FusedSGD(m_n.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    o_r = torch.optim.SGD(m_r.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    ln, lr_ = [], []
    for i in range(3):
        fused.set_backend("native")
        o_n.zero_grad(set_to_none=True)
        loss = fused.softmax_cross_entropy(m_n(xs[i]), ys[i])
        loss.backward()
        o_n.step()
        ln.append(float(loss))
        fused.set_backend("torch")
        o_r.zero_grad(set_to_none=True)
        with chunked_fp32_convs():
            loss = torch.nn.functional.cross_entropy(m_r(_cl(xs[i].float())), ys[i])
        loss.backward()
        o_r.step()
        lr_.append(float(loss))
        torch.cuda.empty_cache()
    fused.set_backend("auto")
    print("native", ln, "fp32", lr_)
    for a, b in zip(ln, lr_):
        assert abs(a - b) / abs(b) < 1e-2, (ln, lr_)
    werr = nrmerr(m_n.fc.weight.detach(), m_r.fc.weight.detach())
    assert werr < 0.02, werr

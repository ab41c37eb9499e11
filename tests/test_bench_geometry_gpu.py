"""Numerics at the benchmark geometry (not only at toy batch sizes).

The native kernels' large-M paths -- 32-bit element offsets in the epilogues and
pooling, split-K weight-gradient slabs, BatchNorm partial-row reductions over
tens of thousands of rows -- only occur at the batch sizes the benchmarks run.
These tests run ResNet blocks at those sizes and compare native bf16 forward and
backward against an fp32 PyTorch reference (inputs rounded to bf16), with the
stock autocast(bf16) error as the yardstick (same rule as
tests/test_kernels_gpu.py::test_resnet50_blocks_native_vs_fp32_reference):
native may not be worse than max(3 x autocast, 0.03) in relative Frobenius norm.

  * ResNet-50, 512 images / GPU at 224x224: stem (conv-BN-ReLU-maxpool node) and
    the first and second block of every stage.
  * ResNet-152 at 1024 images / GPU (the large-batch config): stem and layer1.0
    (M = 1024*112*112 = 12.8 M rows at the stem; 822 M-element activations).
"""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.slow]  # PDT_SLOW_TESTS=1; last run: profiles/bench_geometry_numerics.txt

from pytorch_distributed_template_amd.ops import fused  # noqa: E402
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def nrmerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-6)).item()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def setup_module(module):
    assert no.available(), "native library must be built and loaded on GPU runs"
    no.require()
    torch.backends.cudnn.benchmark = False  # MIOpen immediate mode for the references (no find at bs 512+)


def _run(fn, x, g, params, mode):
    for p in params:
        p.grad = None
    xi = x.detach().clone()
    if mode == "fp32":
        xi = xi.float()
    xi.requires_grad_(True)
    fused.set_backend("native" if mode == "native" else "torch")
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(mode == "autocast")):
            y = fn(xi)
        y.float().backward(g.float() if mode == "fp32" else g.to(y.dtype))
    finally:
        fused.set_backend("auto")
    out = (y.detach().float(), xi.grad.float(), [p.grad.float().clone() for p in params])
    del y, xi
    return out


def _check(name, fn, x, params):
    with torch.no_grad():
        fused.set_backend("torch")
        y0 = fn(x.float()).to(torch.bfloat16)
        fused.set_backend("auto")
    g = _cl(torch.randn(y0.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(5))
            .to(torch.bfloat16))
    yr, dxr, pr = _run(fn, x, g, params, "fp32")
    yn, dxn, pn = _run(fn, x, g, params, "native")
    en = [nrmerr(yn, yr), nrmerr(dxn, dxr)] + [nrmerr(a, b) for a, b in zip(pn, pr)]
    del yn, dxn, pn
    ya, dxa, pa = _run(fn, x, g, params, "autocast")
    ea = [nrmerr(ya, yr), nrmerr(dxa, dxr)] + [nrmerr(a, b) for a, b in zip(pa, pr)]
    del ya, dxa, pa, yr, dxr, pr
    torch.cuda.empty_cache()
    bad = any(e > max(3 * a, 0.03) for e, a in zip(en, ea))
    msg = f"{name}: native {['%.4f' % e for e in en]} autocast {['%.4f' % e for e in ea]}"
    print(msg)
    assert not bad, msg
    return _cl(y0)


def _stem(m):
    return lambda x: fused.conv_bn_relu_maxpool(x, m.conv1, m.bn1)


@pytest.mark.timeout(600)
def test_resnet50_bs512_stem_and_blocks_vs_fp32():
    from pytorch_distributed_template_amd.models import resnet50
    torch.manual_seed(31)
    m = resnet50(num_classes=1000).cuda().to(memory_format=torch.channels_last)
    x = no.synthetic_images((512, 3, 224, 224), torch.bfloat16, torch.device("cuda"), seed=3)
    x = _cl(x)
    x = _check("stem bs512", _stem(m), x, [m.conv1.weight, m.bn1.weight])
    for li, layer in enumerate([m.layer1, m.layer2, m.layer3, m.layer4]):
        for bi in (0, 1):
            blk = layer[bi]
            x = _check(f"layer{li + 1}.{bi} bs512", lambda t, b=blk: fused.bottleneck(t, b), x,
                       [blk.conv1.weight, blk.conv2.weight, blk.conv3.weight, blk.bn3.weight])
        for bi in range(2, len(layer)):  # advance the activations through the rest of the stage
            with torch.no_grad():
                fused.set_backend("native")
                x = _cl(fused.bottleneck(x, layer[bi]))
                fused.set_backend("auto")


@pytest.mark.timeout(600)
def test_resnet152_bs1024_stem_and_layer1_vs_fp32():
    from pytorch_distributed_template_amd.models import resnet152
    torch.manual_seed(32)
    m = resnet152(num_classes=1000).cuda().to(memory_format=torch.channels_last)
    x = _cl(no.synthetic_images((1024, 3, 224, 224), torch.bfloat16, torch.device("cuda"), seed=4))
    x = _check("resnet152 stem bs1024", _stem(m), x, [m.conv1.weight, m.bn1.weight])
    blk = m.layer1[0]
    _check("resnet152 layer1.0 bs1024", lambda t: fused.bottleneck(t, blk), x,
           [blk.conv1.weight, blk.conv2.weight, blk.conv3.weight, blk.bn3.weight])

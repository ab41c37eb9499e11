"""Under backend "native" an op the HIP kernels cannot run is an error, never a silent
stock-PyTorch (MIOpen / SDPA) substitute; under "auto" it warns once and runs the
torch op."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

from pytorch_distributed_template_amd.ops import fused  # noqa: E402
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


@pytest.fixture
def backend():
    old = fused.get_backend()
    yield fused.set_backend
    fused.set_backend(old)


def test_native_backend_raises_on_unsupported_ops(backend):
    backend("native")
    qkv = torch.randn(2, 10, 3 * 4 * 32, device="cuda", dtype=torch.bfloat16)  # head dim 32
    with pytest.raises(NotImplementedError, match="qkv_attention"):
        fused.qkv_attention(qkv, 4)
    conv = nn.Conv2d(16, 32, 3, padding=1, groups=2, bias=False).cuda()  # grouped conv
    bn = nn.BatchNorm2d(32).cuda()
    x = torch.randn(2, 16, 8, 8, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(NotImplementedError, match="conv_bn_act"):
        fused.conv_bn_act(x, conv, bn)
    pe = nn.Conv2d(3, 64, 16, stride=8).cuda()  # overlapping patches
    with pytest.raises(NotImplementedError, match="patch_embed"):
        fused.patch_embed(torch.randn(1, 3, 32, 32, device="cuda", dtype=torch.bfloat16), pe)


def test_auto_backend_warns_and_runs_torch(backend):
    backend("auto")
    no._FALLBACK_WARNED.discard("qkv_attention")
    qkv = torch.randn(2, 10, 3 * 4 * 32, device="cuda", dtype=torch.bfloat16)
    with pytest.warns(UserWarning, match="qkv_attention"):
        o = fused.qkv_attention(qkv, 4)
    assert o.shape == (2, 10, 128)


def test_attention_entry_runs_the_fused_kernel(backend):
    """fused.attention on [B, H, T, 64] packs q/k/v for the native kernel (no SDPA)."""
    backend("native")
    q, k, v = (torch.randn(2, 3, 50, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    o = fused.attention(q, k, v)
    ref = torch.nn.functional.scaled_dot_product_attention(q.float(), k.float(), v.float())
    assert o.shape == ref.shape
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)

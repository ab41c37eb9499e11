"""Native MnistModel (csrc/lenet.hip: whole-network forward / backward kernels) and
the NLL loss kernels against a float64 PyTorch reference of the reference model
(/root/reference/model/model.py:15-22, /root/reference/model/loss.py:4-5), with the
dropout masks the kernel drew fed to the reference so training mode is compared
exactly."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from pytorch_distributed_template_amd.models import MnistModel  # noqa: E402
from pytorch_distributed_template_amd.ops import fused  # noqa: E402
from pytorch_distributed_template_amd.ops import native_ops as no  # noqa: E402


def setup_module(module):
    assert no.available(), "native library must be built and loaded on GPU runs"
    no.require()
    fused.set_backend("native")


def teardown_module(module):
    fused.set_backend("auto")


def _ref_logp(model, x, m2=None, m1=None, p2=0.5, p1=0.5):
    """float64 CPU reference of MnistModel.forward with explicit dropout masks."""
    P = {k: v.detach().double().cpu() for k, v in model.state_dict().items()}
    x = x.double().cpu()
    h = F.max_pool2d(F.conv2d(x, P["conv1.weight"], P["conv1.bias"]), 2).relu()
    c = F.conv2d(h, P["conv2.weight"], P["conv2.bias"])
    if m2 is not None:
        c = c * (m2.double().cpu() / (1 - p2))[:, :, None, None]
    h = F.max_pool2d(c, 2).relu().flatten(1)
    z = F.linear(h, P["fc1.weight"], P["fc1.bias"]).relu()
    if m1 is not None:
        z = z * (m1.double().cpu() / (1 - p1))
    return F.log_softmax(F.linear(z, P["fc2.weight"], P["fc2.bias"]), 1)


def _model(seed=0):
    torch.manual_seed(seed)
    return MnistModel().cuda()


def test_lenet_eval_forward_matches_fp64_reference():
    m = _model().eval()
    x = torch.randn(64, 1, 28, 28, device="cuda")
    out = m(x)
    assert out.shape == (64, 10) and out.dtype == torch.float32
    ref = _ref_logp(m, x)
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-4, atol=1e-4)


def test_lenet_train_forward_backward_matches_reference_with_same_masks():
    m = _model(1).train()
    B = 96
    x = torch.randn(B, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    m2 = torch.empty((B, 20), dtype=torch.uint8, device="cuda")
    m1 = torch.empty((B, 50), dtype=torch.uint8, device="cuda")
    logp = no.lenet_forward(m, x, masks=(m2, m1), seed=1234)
    loss = no.nll_loss(logp, y)
    loss.backward()
    # masks: Bernoulli(0.5) per (image, unit), not all equal
    assert 0.3 < m2.float().mean().item() < 0.7 and 0.3 < m1.float().mean().item() < 0.7

    ref_m = MnistModel().double()
    ref_m.load_state_dict({k: v.double().cpu() for k, v in m.state_dict().items()})
    ref = _ref_logp(ref_m, x, m2, m1)
    torch.testing.assert_close(logp.detach().double().cpu(), ref, rtol=1e-4, atol=1e-4)

    # autograd reference of the same function in float64
    P = {k: v.detach().double().cpu().requires_grad_(True) for k, v in m.state_dict().items()}
    xc = x.double().cpu()
    h = F.max_pool2d(F.conv2d(xc, P["conv1.weight"], P["conv1.bias"]), 2).relu()
    c = F.conv2d(h, P["conv2.weight"], P["conv2.bias"]) * (m2.double().cpu() * 2)[:, :, None, None]
    h = F.max_pool2d(c, 2).relu().flatten(1)
    z = F.linear(h, P["fc1.weight"], P["fc1.bias"]).relu() * (m1.double().cpu() * 2)
    lp = F.log_softmax(F.linear(z, P["fc2.weight"], P["fc2.bias"]), 1)
    rl = F.nll_loss(lp, y.cpu())
    rl.backward()
    torch.testing.assert_close(loss.detach().double().cpu(), rl.detach(), rtol=1e-5, atol=1e-6)
    for name, prm in m.named_parameters():
        g = prm.grad.double().cpu()
        r = P[name].grad
        err = ((g - r).norm() / r.norm().clamp_min(1e-12)).item()
        assert err < 1e-4, (name, err)


def test_lenet_same_seed_same_masks_and_eval_has_none():
    m = _model(2).train()
    x = torch.randn(8, 1, 28, 28, device="cuda")
    a = no.lenet_forward(m, x, seed=7)
    b = no.lenet_forward(m, x, seed=7)
    c = no.lenet_forward(m, x, seed=8)
    assert torch.equal(a, b) and not torch.equal(a, c)
    m.eval()
    torch.testing.assert_close(m(x), no.lenet_forward(m, x))


def test_nll_loss_kernels_match_torch():
    B, C = 300, 10
    logp = torch.log_softmax(torch.randn(B, C, device="cuda"), 1).requires_grad_(True)
    y = torch.randint(0, C, (B,), device="cuda")
    y[::7] = -100  # ignore_index
    loss = no.nll_loss(logp, y)
    loss.backward()
    g = logp.grad.clone()
    logp.grad = None
    ref = F.nll_loss(logp, y)
    ref.backward()
    torch.testing.assert_close(loss, ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(g, logp.grad, rtol=1e-6, atol=1e-7)


def test_nll_loss_out_of_range_target_fails_loudly(monkeypatch):
    """torch's F.nll_loss raises on a target outside [0, C); the native kernel cannot
    raise from the device: the batch's loss is NaN, and the next call (lazy check, no
    sync in the step) or this call (PDT_CHECK_TARGETS=sync) raises."""
    B, C = 64, 10
    logp = torch.log_softmax(torch.randn(B, C, device="cuda"), 1)
    y = torch.randint(0, C, (B,), device="cuda")
    y[5] = C  # == num_classes: out of range
    loss = no.nll_loss(logp, y)
    assert torch.isnan(loss).item()
    torch.cuda.synchronize()
    with pytest.raises(ValueError, match="out of range"):
        no.nll_loss(logp, torch.randint(0, C, (B,), device="cuda"))
    monkeypatch.setenv("PDT_CHECK_TARGETS", "sync")
    with pytest.raises(ValueError, match="out of range"):
        no.nll_loss(logp, y)
    ok = no.nll_loss(logp, torch.randint(0, C, (B,), device="cuda"))
    assert torch.isfinite(ok).item()


def test_mnist_config_step_uses_native_path():
    from pytorch_distributed_template_amd.models import loss as L
    m = _model(3).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, amsgrad=True)
    # a learnable task (noisy class prototypes): random labels on random images with
    # dropout 0.5 barely move in a few dozen steps (stock torch drops to ~0.42x in 40)
    g = torch.Generator().manual_seed(5)
    proto = torch.randn(10, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (128,), generator=g)
    x = (proto[y] + 0.5 * torch.randn(128, 1, 28, 28, generator=g)).cuda()
    y = y.cuda()
    losses = []
    for _ in range(40):
        opt.zero_grad()
        out = m(x)
        assert out.grad_fn is not None and "LeNet" in type(out.grad_fn).__name__
        loss = L.nll_loss(out, y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] * 0.7, losses


def test_config_adam_becomes_fused_on_gpu_and_matches_torch():
    """The reference config's "Adam" runs as FusedAdam on the native GPU path (one HIP
    launch per step) and tracks torch.optim.Adam(amsgrad) on the same gradients."""
    from pytorch_distributed_template_amd.optim import FusedAdam
    from pytorch_distributed_template_amd.runtime.builder import build_optimizer
    from test_optim_cpu import _mnist_opt_cfg
    torch.manual_seed(0)
    a = _model(3)
    b = _model(3)
    b.load_state_dict(a.state_dict())
    oa, _ = build_optimizer(_mnist_opt_cfg(), a)
    ob = torch.optim.Adam(b.parameters(), lr=1e-3, weight_decay=0, amsgrad=True)
    assert isinstance(oa, FusedAdam) and not oa.write_bf16_shadow
    for _ in range(5):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            for p in m.parameters():
                p.grad = torch.sin(p.detach() * 3.0 + 1.0)
            o.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6)
    assert set(oa.state_dict()["state"][0]) == set(ob.state_dict()["state"][0])

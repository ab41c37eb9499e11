import torch

from pytorch_distributed_template_amd.models import MnistModel, ResNet50, ResNet152, ViT_B_16, resnet50
from pytorch_distributed_template_amd.models import loss as L, metric as Mt
from pytorch_distributed_template_amd.ops import fused


def test_param_counts_match_survey():
    # SURVEY §2.1 C10, §2.6(b)
    assert sum(p.numel() for p in MnistModel().parameters()) == 21840
    assert sum(p.numel() for p in ResNet50().parameters()) == 25557032
    assert sum(p.numel() for p in ResNet152().parameters()) == 60192808
    assert sum(p.numel() for p in ViT_B_16().parameters()) == 86567656


def test_base_model_str():
    assert str(MnistModel()).endswith("Trainable parameters: 21840")


def test_mnist_forward_logprobs():
    m = MnistModel().eval()
    out = m(torch.randn(3, 1, 28, 28))
    assert out.shape == (3, 10)
    assert torch.allclose(out.exp().sum(1), torch.ones(3), atol=1e-5)


def test_resnet_torch_path_backward_cpu():
    fused.set_backend("torch")
    m = resnet50(num_classes=10)
    x = torch.randn(2, 3, 64, 64)
    loss = L.cross_entropy(m(x), torch.tensor([1, 2]))
    loss.backward()
    assert m.conv1.weight.grad is not None and torch.isfinite(loss)
    fused.set_backend("auto")


def test_vit_small_forward_backward_cpu():
    from pytorch_distributed_template_amd.models.vit import VisionTransformer
    m = VisionTransformer(image_size=32, patch_size=8, embed_dim=64, depth=2, num_heads=4, num_classes=7)
    out = m(torch.randn(2, 3, 32, 32))
    assert out.shape == (2, 7)
    out.sum().backward()


def test_metrics():
    out = torch.tensor([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1]])
    t = torch.tensor([1, 2])
    assert Mt.accuracy(out, t) == 0.5
    assert Mt.top_k_acc(out, t, k=2) == 0.5
    assert Mt.top_k_acc(out, t, k=3) == 1.0
    assert int(Mt.correct_count(out, t)) == 1


def test_losses():
    lp = torch.log_softmax(torch.randn(4, 5), 1)
    t = torch.tensor([0, 1, 2, 3])
    assert torch.allclose(L.nll_loss(lp, t), torch.nn.functional.nll_loss(lp, t))
    lg = torch.randn(4, 5)
    assert torch.allclose(L.cross_entropy(lg, t), torch.nn.functional.cross_entropy(lg, t))

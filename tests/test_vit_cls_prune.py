"""The last ViT block computed for the class token's row only (models/vit.py Block._forward_cls):
the classifier reads token 0 alone, so the model output and every parameter gradient must equal
those of the full block (torch path on CPU here; the native fp8 path in
tests/test_vit_fusion_gpu.py::test_vit_cls_prune_native_matches_full)."""
import torch

from pytorch_distributed_template_amd.models.vit import VisionTransformer


def test_cls_prune_same_output_and_grads_cpu():
    torch.manual_seed(0)
    m = VisionTransformer(image_size=32, patch_size=8, embed_dim=128, depth=3, num_heads=2, num_classes=10)
    x = torch.randn(4, 3, 32, 32)
    res = {}
    for prune in (False, True):
        m.zero_grad(set_to_none=True)
        m.cls_prune = prune
        y = m(x)
        torch.nn.functional.cross_entropy(y, torch.arange(4)).backward()
        res[prune] = (y.detach(), {n: p.grad.clone() for n, p in m.named_parameters()})
    torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-5, atol=1e-5)
    for n, g in res[False][1].items():
        torch.testing.assert_close(res[True][1][n], g, rtol=1e-4, atol=1e-6, msg=n)

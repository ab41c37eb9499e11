"""Model registry (``arch.type`` in config). Reference: ``/root/reference/model/model.py``."""
from .mnist import MnistModel  # noqa: F401
from .resnet import ResNet, ResNet50, ResNet101, ResNet152, resnet50, resnet101, resnet152  # noqa: F401
from .vit import VisionTransformer, ViT_B_16, vit_b_16  # noqa: F401

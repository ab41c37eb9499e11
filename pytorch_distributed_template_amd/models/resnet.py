"""ResNet-50/101/152 (v1.5: stride on the 3x3 conv) for MI355X.

Not present in the reference (its only model is the LeNet at
``/root/reference/model/model.py:6-22``); the BASELINE north-star adds
ResNet-50/152 on synthetic 3x224x224 data.

Design (MI355X-first, not a torchvision translation):
  * activations are NHWC (``channels_last``) bf16 end to end -- the layout
    the implicit-GEMM conv kernels in ``csrc/conv_igemm.hip`` read with
    K(=Cin) contiguous, 128-byte rows per MFMA K-step;
  * every conv is followed by a fused BatchNorm(+residual)(+ReLU) unit
    (``ops.conv_bn_act``) so the memory-bound BN/ReLU/add passes are one
    read + one write of the activation instead of four;
  * parameter names follow the familiar ``conv1/bn1/layerX.Y.convZ/...``
    scheme so state_dicts are interchangeable with other ResNet code.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..base.base_model import BaseModel
from ..ops import fused


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: bool = False):
        super().__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        if downsample:
            self.downsample = nn.Sequential(
                nn.Conv2d(inplanes, planes * self.expansion, 1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * self.expansion),
            )
        else:
            self.downsample = None

    def forward(self, x):
        # conv-BN-ReLU x3 with BN3 + residual add + ReLU in one pass; on the
        # native path the whole block is one autograd node (ops.native_ops._Bottleneck)
        return fused.bottleneck(x, self)


class ResNet(BaseModel):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000, zero_init_residual: bool = False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)

        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def _make_layer(self, planes, blocks, stride=1):
        layers = [Bottleneck(self.inplanes, planes, stride,
                             downsample=(stride != 1 or self.inplanes != planes * Bottleneck.expansion))]
        self.inplanes = planes * Bottleneck.expansion
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = fused.conv_bn_relu_maxpool(x, self.conv1, self.bn1, 3, 2, 1)
        # all 16 (50) bottlenecks as one chain: on the native path each block's output BN
        # pass runs inside the next block's conv1 (ops.native_ops.bottleneck_chain); the
        # layerN containers keep the usual state_dict names
        x = fused.bottleneck_chain(x, [*self.layer1, *self.layer2, *self.layer3, *self.layer4])
        x = fused.global_avg_pool(x)
        return fused.linear(x, self.fc)


def resnet50(num_classes: int = 1000, **kw):
    return ResNet((3, 4, 6, 3), num_classes=num_classes, **kw)


def resnet101(num_classes: int = 1000, **kw):
    return ResNet((3, 4, 23, 3), num_classes=num_classes, **kw)


def resnet152(num_classes: int = 1000, **kw):
    return ResNet((3, 8, 36, 3), num_classes=num_classes, **kw)


# Config-registry names (``arch.type`` in config JSON)
class ResNet50(ResNet):
    def __init__(self, num_classes: int = 1000, **kw):
        super().__init__((3, 4, 6, 3), num_classes=num_classes, **kw)


class ResNet101(ResNet):
    def __init__(self, num_classes: int = 1000, **kw):
        super().__init__((3, 4, 23, 3), num_classes=num_classes, **kw)


class ResNet152(ResNet):
    def __init__(self, num_classes: int = 1000, **kw):
        super().__init__((3, 8, 36, 3), num_classes=num_classes, **kw)

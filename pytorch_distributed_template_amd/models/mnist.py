"""LeNet-style MNIST demo model (reference: ``/root/reference/model/model.py:6-22``).

Same layers and parameter names (conv1 1->10 k5, conv2 10->20 k5, channel
dropout, fc1 320->50, fc2 50->classes, log-softmax output; 21,840 params),
so state_dicts line up with the reference's ``MnistModel``.

On an MI355X the whole network runs as two hand-written kernels (forward, and a
backward that recomputes the forward in LDS: ``csrc/lenet.hip``) instead of
~45 stock-op launches; on CPU (gloo plumbing) it is plain torch ops.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..base.base_model import BaseModel


class MnistModel(BaseModel):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 10, kernel_size=5)
        self.conv2 = nn.Conv2d(10, 20, kernel_size=5)
        self.conv2_drop = nn.Dropout2d()
        self.fc1 = nn.Linear(20 * 4 * 4, 50)
        self.fc2 = nn.Linear(50, num_classes)

    def forward(self, x):
        from ..ops import fused
        if fused.use_native(x):
            from ..ops import native_ops
            if native_ops.lenet_supported(self, x) and not x.requires_grad:
                return native_ops.lenet_forward(self, x)
            native_ops.fallback("MnistModel", f"input {tuple(x.shape)} requires_grad={x.requires_grad} "
                                              "(kernel: [B, 1, 28, 28], the reference layer sizes)")
        h = F.max_pool2d(self.conv1(x), 2).relu()
        h = F.max_pool2d(self.conv2_drop(self.conv2(h)), 2).relu()
        h = torch.flatten(h, 1)
        h = F.dropout(self.fc1(h).relu(), training=self.training)
        return F.log_softmax(self.fc2(h), dim=1)

"""Loss registry (``"loss"`` key in config). Reference: ``/root/reference/model/loss.py:4-5``.

``cross_entropy`` routes to the fused softmax-cross-entropy HIP kernel
(``csrc/xent.hip``) for GPU tensors; ``nll_loss`` matches the reference (model
emits log-probabilities) and runs the ``csrc/lenet.hip`` NLL kernels on GPU.
"""
import torch
import torch.nn.functional as F

from ..ops import fused


def nll_loss(output, target):
    if fused.use_native(output):
        from ..ops import native_ops
        if output.dim() == 2 and output.dtype == torch.float32:
            return native_ops.nll_loss(output, target)
        native_ops.fallback("nll_loss", f"{tuple(output.shape)} {output.dtype} (kernel: fp32 [B, C])")
    return F.nll_loss(output, target)


def cross_entropy(output, target):
    return fused.softmax_cross_entropy(output, target)


def label_smoothing_cross_entropy(output, target, smoothing=0.1):
    return fused.softmax_cross_entropy(output, target, label_smoothing=smoothing)

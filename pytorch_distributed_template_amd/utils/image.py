"""Tiny ``make_grid`` (torchvision is not installed; the reference used
``torchvision.utils.make_grid`` for TensorBoard image logging at
``trainer/trainer.py:69``)."""
import math

import torch


def make_grid(tensor: torch.Tensor, nrow: int = 8, padding: int = 2, normalize: bool = False) -> torch.Tensor:
    if tensor.dim() == 3:
        tensor = tensor.unsqueeze(0)
    tensor = tensor.float()
    if tensor.shape[1] == 1:
        tensor = tensor.repeat(1, 3, 1, 1)
    if normalize:
        lo, hi = tensor.min(), tensor.max()
        tensor = (tensor - lo) / (hi - lo).clamp_min(1e-5)
    n, c, h, w = tensor.shape
    xmaps = min(nrow, n)
    ymaps = int(math.ceil(n / xmaps))
    H, W = h + padding, w + padding
    grid = tensor.new_zeros((c, ymaps * H + padding, xmaps * W + padding))
    for k in range(n):
        y, x = divmod(k, xmaps)
        grid[:, y * H + padding: y * H + padding + h, x * W + padding: x * W + padding + w] = tensor[k]
    return grid

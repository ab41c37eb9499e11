"""BaseModel (reference: ``/root/reference/base/base_model.py:6-25``).

``__str__`` appends ``Trainable parameters: N`` -- that is what
``logger.info(model)`` prints at startup (``train.py:64-65`` in the reference).
"""
from abc import abstractmethod

import torch.nn as nn


class BaseModel(nn.Module):
    """Base class for all models."""

    @abstractmethod
    def forward(self, *inputs):
        raise NotImplementedError

    def num_trainable_parameters(self) -> int:
        return int(sum(p.numel() for p in self.parameters() if p.requires_grad))

    def __str__(self):
        return super().__str__() + "\nTrainable parameters: {}".format(self.num_trainable_parameters())

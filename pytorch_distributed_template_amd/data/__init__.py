"""Data loader registry (``*_loader.type`` in config).

Reference: ``/root/reference/data_loader/data_loaders.py`` (MnistDataLoader).
"""
from .mnist import MnistDataLoader, MnistDataset, read_idx, synthetic_mnist  # noqa: F401
from .samplers import EvalShardSampler, shard_bounds  # noqa: F401
from .synthetic import (SyntheticImageDataset, SyntheticImageLoader, SyntheticImageNet,  # noqa: F401
                        SyntheticImageNetLoader)

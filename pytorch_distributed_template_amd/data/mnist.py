"""MNIST demo loader (reference: ``/root/reference/data_loader/data_loaders.py:8-27``).

Same constructor signature and semantics as the reference's
``MnistDataLoader(data_dir, batch_size, shuffle=True, num_workers=1,
training=True)``: ToTensor + Normalize(0.1307, 0.3081), a distributed sampler
when the world is larger than one.

Differences (the GPU boxes have no network and torchvision is absent):
  * the dataset is read directly from the IDX files torchvision would have
    downloaded (``<data_dir>/MNIST/raw/`` or ``<data_dir>/``, plain or ``.gz``)
    and normalised once, as one tensor, instead of per sample through PIL;
  * if the files are missing, a deterministic synthetic stand-in of
    ``synthetic_size`` samples is used (class prototypes + noise, so the demo
    model still learns); the log says which one was loaded;
  * the training sampler is ``set_epoch``-ed every epoch (Q6) and evaluation
    shards are unpadded (Q9), see ``samplers.py``.
"""
from __future__ import annotations

import gzip
import logging
from pathlib import Path

import numpy as np
import torch
from torch.utils.data import Dataset
from torch.utils.data.distributed import DistributedSampler

from ..base import BaseDataLoader
from ..utils import dist as pdist
from .samplers import EvalShardSampler

MNIST_MEAN, MNIST_STD = 0.1307, 0.3081
_FILES = {True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
          False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}


def read_idx(path: Path) -> np.ndarray:
    """Parse an IDX file (big-endian header: 0,0,dtype,ndim, then ndim uint32 dims)."""
    raw = path.read_bytes()
    if path.suffix == ".gz":
        raw = gzip.decompress(raw)
    if len(raw) < 4 or raw[0] != 0 or raw[1] != 0:
        raise ValueError(f"{path}: not an IDX file")
    code, ndim = raw[2], raw[3]
    dtypes = {0x08: np.uint8, 0x09: np.int8, 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4", 0x0E: ">f8"}
    dims = np.frombuffer(raw, dtype=">u4", count=ndim, offset=4).astype(np.int64)
    return np.frombuffer(raw, dtype=dtypes[code], offset=4 + 4 * ndim).reshape(dims)


def _find(data_dir: Path, stem: str):
    for d in (data_dir / "MNIST" / "raw", data_dir):
        for name in (stem, stem + ".gz"):
            if (d / name).is_file():
                return d / name
    return None


def synthetic_mnist(n: int, training: bool, seed: int = 0):
    """Deterministic MNIST-shaped stand-in: uint8 [n,28,28] and int64 [n] labels.
    Prototypes are shared by every split (same ``seed``), samples differ."""
    g = torch.Generator().manual_seed(seed)
    protos = (torch.rand(10, 28, 28, generator=g) > 0.7).float() * 200.0
    g.manual_seed(seed + (1 if training else 2))
    labels = torch.randint(0, 10, (n,), generator=g)
    imgs = protos[labels] + torch.randn(n, 28, 28, generator=g) * 40.0
    return imgs.clamp_(0, 255).to(torch.uint8), labels


class MnistDataset(Dataset):
    """Normalised MNIST images held as one float tensor [N,1,28,28] (+ int64 targets)."""

    def __init__(self, data_dir, training=True, synthetic_size=None):
        data_dir = Path(data_dir)
        img_f, lbl_f = (_find(data_dir, s) for s in _FILES[training])
        if img_f is not None and lbl_f is not None:
            imgs = torch.from_numpy(read_idx(img_f).copy())
            labels = torch.from_numpy(read_idx(lbl_f).astype(np.int64))
            self.source = str(img_f.parent)
        else:
            n = synthetic_size or (60000 if training else 10000)
            imgs, labels = synthetic_mnist(n, training)
            self.source = "synthetic"
        self.data = ((imgs.float() / 255.0 - MNIST_MEAN) / MNIST_STD).unsqueeze(1).contiguous()
        self.targets = labels

    def __len__(self):
        return self.targets.shape[0]

    def __getitem__(self, i):
        return self.data[i], self.targets[i]


def _batch_collate(batch):
    xs, ys = zip(*batch)
    return torch.stack(xs), torch.stack(ys)


class MnistDataLoader(BaseDataLoader):
    """MNIST data loading demo using BaseDataLoader."""

    def __init__(self, data_dir, batch_size, shuffle=True, num_workers=1, training=True, synthetic_size=None):
        self.data_dir = data_dir
        self.dataset = MnistDataset(data_dir, training=training, synthetic_size=synthetic_size)
        logging.getLogger("data").debug("MNIST (%s): %d samples", self.dataset.source, len(self.dataset))
        if pdist.get_world_size() > 1:
            sampler = (DistributedSampler(self.dataset, shuffle=shuffle) if training
                       else EvalShardSampler(self.dataset))
        else:
            sampler = None
        super().__init__(self.dataset, batch_size, shuffle, num_workers, collate_fn=_batch_collate,
                         sampler=sampler)

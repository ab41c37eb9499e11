"""Device-resident synthetic ImageNet-shaped data (BASELINE configs 2-5).

Not in the reference (its only dataset is torchvision MNIST,
``/root/reference/data_loader/data_loaders.py:22``); the north-star benchmarks
run on synthetic 3x224x224 images with random labels.

MI355X-first design: a pool of ``pool`` batches is generated ONCE, on the GPU,
by the native counter-based fill kernel (``csrc/misc.hip``,
``pdt_fill_uniform_bf16``), already bf16 and NHWC (``channels_last``) -- the
layout the implicit-GEMM conv kernels read. Iterating hands out those
resident tensors round-robin, so the hot loop has no H2D copy, no host
collate and no worker processes (the reference's per-step pageable H2D copy,
SURVEY Q11/§7.4-8). 256 images x 3x224x224 bf16 is 77 MB per pooled batch,
noise next to 288 GB of HBM3E.

Sharding follows ``samplers.py``: in training every rank sees
``ceil(num_samples / world)`` samples (DistributedSampler padding); in
evaluation the shards are contiguous and unpadded, so the per-rank counts sum
to ``num_samples`` exactly.
"""
from __future__ import annotations

import math

import torch

from ..utils import dist as pdist
from .samplers import shard_bounds

_DTYPES = {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float32": torch.float32, "fp32": torch.float32,
           "float16": torch.float16, "fp16": torch.float16}


def _default_device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class SyntheticImageDataset:
    """Stands in for ``loader.dataset`` (``len()`` = the global sample count)."""

    def __init__(self, num_samples, image_size, num_classes):
        self.num_samples = int(num_samples)
        self.image_size = image_size
        self.num_classes = num_classes

    def __len__(self):
        return self.num_samples


class SyntheticImageLoader:
    """Iterable of ``(images, labels)`` device tensors.

    images: [B, 3, H, W] in ``dtype`` (NHWC strides when ``channels_last``),
    uniform in [-1, 1); labels: int64 [B] in [0, num_classes).
    """

    def __init__(self, batch_size, num_samples=1281167, dtype=None, pool=2, device=None, image_size=224,
                 num_classes=1000, channels=3, channels_last=True, training=True, seed=0):
        self.batch_size = int(batch_size)
        self.device = torch.device(device) if device is not None else _default_device()
        if dtype is None:
            dtype = "bfloat16" if self.device.type == "cuda" else "float32"
        self.dtype = _DTYPES[dtype] if isinstance(dtype, str) else dtype
        self.dataset = SyntheticImageDataset(num_samples, image_size, num_classes)
        self.training = training
        rank, world = pdist.get_rank(), pdist.get_world_size()
        if training:
            self.n_samples = math.ceil(len(self.dataset) / world)
        else:
            lo, hi = shard_bounds(len(self.dataset), rank, world)
            self.n_samples = hi - lo
        self.epoch = 0
        shape = (self.batch_size, channels, image_size, image_size)
        self._pool = []
        for i in range(max(1, int(pool))):
            bseed = (seed * 1000003 + rank * 7919 + i * 104729 + (0 if training else 15485863)) & 0x7FFFFFFF
            self._pool.append((self._images(shape, channels_last, bseed), self._labels(num_classes, bseed)))

    def _images(self, shape, channels_last, seed):
        fmt = torch.channels_last if channels_last else torch.contiguous_format
        if self.device.type == "cuda":
            from ..ops import native_ops
            if native_ops.available():
                B, C, H, W = shape
                if channels_last and self.dtype == torch.bfloat16 and C % 4:
                    # NHWC with the channel dim zero-padded to 4 in storage: the images are the
                    # [B, C, H, W] view, and the space-to-depth stem GEMM reads 16-B chunks of two
                    # padded pixels in place (no per-step pad copy; ops.native_ops.nhwc_padded_view)
                    cp = (C + 3) // 4 * 4
                    buf = torch.empty((B, H, W, cp), dtype=torch.bfloat16, device=self.device)
                    native_ops.fill_uniform_(buf, seed)
                    buf[..., C:] = 0
                    x = buf[..., :C].permute(0, 3, 1, 2)
                    x.pdt_nhwc_pad = cp
                    return x
                x = torch.empty(shape, dtype=torch.bfloat16, device=self.device, memory_format=fmt)
                native_ops.fill_uniform_(x, seed)
                return x if self.dtype == torch.bfloat16 else x.to(self.dtype)
        g = torch.Generator().manual_seed(seed)
        x = torch.rand(shape, generator=g).mul_(2).sub_(1)
        return x.to(self.device, self.dtype).contiguous(memory_format=fmt)

    def _labels(self, num_classes, seed):
        g = torch.Generator().manual_seed(seed)
        return torch.randint(0, num_classes, (self.batch_size,), generator=g).to(self.device)

    def __len__(self):
        return math.ceil(self.n_samples / self.batch_size)

    def __iter__(self):
        n_pool = len(self._pool)
        off = self.epoch % n_pool if self.training else 0
        left = self.n_samples
        for i in range(len(self)):
            x, y = self._pool[(i + off) % n_pool]
            if left < self.batch_size:
                x, y = x[:left], y[:left]
            left -= self.batch_size
            yield x, y

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)


class SyntheticImageNetLoader(SyntheticImageLoader):
    """Config-facing name (``train_loader.type``). Accepts the reference loader
    keys (``data_dir``, ``shuffle``, ``num_workers``) for schema compatibility;
    they have no effect on device-resident synthetic data."""

    def __init__(self, batch_size, num_samples=1281167, pool=2, data_dir=None, shuffle=True, num_workers=0,
                 training=True, dtype=None, image_size=224, num_classes=1000, channels_last=True, seed=0):
        super().__init__(batch_size, num_samples=num_samples, dtype=dtype, pool=pool, image_size=image_size,
                         num_classes=num_classes, channels_last=channels_last, training=training, seed=seed)

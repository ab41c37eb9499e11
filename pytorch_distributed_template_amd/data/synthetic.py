"""Synthetic ImageNet-shaped data (BASELINE configs 2-5).

Not in the reference (its only dataset is torchvision MNIST,
``/root/reference/data_loader/data_loaders.py:22``); the north-star benchmarks
run on synthetic 3x224x224 images with random labels. Two loaders:

* :class:`SyntheticImageNetLoader` (the config default) is the reference's data
  path: an index-addressable :class:`SyntheticImageNet` dataset -- sample ``i``
  is a pure function of ``(seed, i)`` -- sharded by ``DistributedSampler`` in
  training (``set_epoch`` reshuffles every epoch) and by the unpadded
  :class:`EvalShardSampler` in evaluation, batched by :class:`BaseDataLoader`
  (/root/reference/base/base_data_loader.py:11-19,
  /root/reference/data_loader/data_loaders.py:23-26). MI355X-first: the
  DataLoader moves only the INDEX batch; ``__getitems__`` + ``collate`` turn it
  into images with one HIP launch (``csrc/misc.hip`` ``pdt_synth_images_bf16``)
  that writes bf16 NHWC straight into HBM -- no per-sample host work, no H2D
  image copy, no worker processes. The CPU path computes the same hash in torch
  integer ops, so both devices produce bit-identical samples.
* :class:`SyntheticImageLoader` (``mode: "pool"``) generates ``pool`` batches
  once and hands them out round-robin: the fastest possible feed, kept for
  kernel-level benchmarks (``bench.py --data pool``).

3-channel images on the native path live in NHWC storage zero-padded to 4
channels (the space-to-depth stem GEMM reads 16-B pairs of pixels in place);
the ``[B, 3, H, W]`` tensor is a view into it tagged ``pdt_nhwc_pad``.
"""
from __future__ import annotations

import math

import torch

from torch.utils.data import Dataset, DistributedSampler

from ..base import BaseDataLoader
from ..utils import dist as pdist
from .samplers import EvalShardSampler, shard_bounds

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


_M32 = 0xFFFFFFFF


def _hash32(x: torch.Tensor) -> torch.Tensor:
    """csrc/misc.hip ``hash32`` on int64 tensors holding uint32 values (wrapping products)."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


class SyntheticImageNet(Dataset):
    """Index-addressable synthetic ImageNet: ``self[i]`` = (image_i, label_i), each a pure
    function of ``(seed, i)`` -- uniform [-1, 1) pixels and a label in [0, num_classes).

    ``__getitems__`` (the DataLoader's batched fetch) returns the index list itself;
    :meth:`collate` materialises the whole batch at once on ``device``."""

    def __init__(self, num_samples, image_size=224, num_classes=1000, channels=3, seed=0, device=None,
                 dtype=None, channels_last=True):
        self.num_samples = int(num_samples)
        self.image_size = int(image_size)
        self.num_classes = int(num_classes)
        self.channels = int(channels)
        self.seed = int(seed) & 0x7FFFFFFF
        self.device = torch.device(device) if device is not None else _default_device()
        if dtype is None:
            dtype = "bfloat16" if self.device.type == "cuda" else "float32"
        self.dtype = _DTYPES[dtype] if isinstance(dtype, str) else dtype
        self.channels_last = channels_last

    def __len__(self):
        return self.num_samples

    def __getitem__(self, i):
        x, y = self.collate([int(i)])
        return x[0], y[0]

    def __getitems__(self, indices):
        return list(indices)

    def _native(self) -> bool:
        if self.device.type != "cuda" or self.dtype != torch.bfloat16 or not self.channels_last:
            return False
        from ..ops import native_ops
        return native_ops.available()

    def collate(self, indices):
        """(images [B, C, H, W], labels int64 [B]) for a list of sample indices."""
        B, C, H = len(indices), self.channels, self.image_size
        idx = torch.as_tensor(indices, dtype=torch.int64)
        if self._native():
            from ..ops import native_ops
            cp = (C + 3) // 4 * 4
            buf = torch.empty((B, H, H, cp), dtype=torch.bfloat16, device=self.device)
            y = torch.empty(B, dtype=torch.int64, device=self.device)
            native_ops.synthetic_images_at(buf, idx.to(self.device, non_blocking=True), C, self.seed, y,
                                           self.num_classes)
            x = buf[..., :C].permute(0, 3, 1, 2)
            if cp != C:
                x.pdt_nhwc_pad = cp
            return x, y
        # host path: the kernel's hash in torch integer ops (bit-identical samples)
        s = _hash32(((idx & _M32) * 0x9E3779B9 & _M32) ^ self.seed)                # [B]
        e = torch.arange(H * H * C, dtype=torch.int64)                                # p * C + c
        h = _hash32(((e * 0x85EBCA6B) & _M32)[None, :] ^ s[:, None])
        f = (h >> 8).to(torch.float32) * (2.0 / 16777216.0) - 1.0
        x = f.view(B, H, H, C).permute(0, 3, 1, 2).to(self.dtype)
        if self.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        else:
            x = x.contiguous()
        y = _hash32(((idx & _M32) * 0xC2B2AE35 & _M32) ^ self.seed ^ 0x5BD1E995) % self.num_classes
        return x.to(self.device), y.to(self.device)


class SyntheticImageNetLoader(BaseDataLoader):
    """Config-facing loader (``train_loader.type``): :class:`SyntheticImageNet` through
    ``DistributedSampler`` (training: shuffled, padded to equal per-rank steps,
    ``set_epoch`` reshuffles) or :class:`EvalShardSampler` (evaluation: contiguous,
    unpadded shards), batched by :class:`BaseDataLoader`. Accepts the reference loader
    keys (``data_dir``, ``num_workers``) for schema compatibility; ``pool`` is only read
    by ``mode: "pool"`` (the pooled fast path, :class:`SyntheticImageLoader`)."""

    def __new__(cls, *args, mode="sampler", **kwargs):
        if mode == "pool":
            kw = {k: v for k, v in kwargs.items() if k not in ("data_dir", "shuffle", "num_workers")}
            return SyntheticImageLoader(*args, **kw)
        if mode != "sampler":
            raise ValueError(f"SyntheticImageNetLoader mode must be 'sampler' or 'pool', got {mode!r}")
        return super().__new__(cls)

    def __init__(self, batch_size, num_samples=1281167, pool=2, data_dir=None, shuffle=True, num_workers=0,
                 training=True, dtype=None, image_size=224, num_classes=1000, channels_last=True, seed=0,
                 mode="sampler", device=None):
        self.dataset = SyntheticImageNet(num_samples, image_size=image_size, num_classes=num_classes,
                                         seed=seed + (0 if training else 15485863), device=device, dtype=dtype,
                                         channels_last=channels_last)
        self.training = training
        rank, world = pdist.get_rank(), pdist.get_world_size()
        if training:
            sampler = DistributedSampler(self.dataset, num_replicas=world, rank=rank, shuffle=shuffle, seed=seed)
        else:
            sampler = EvalShardSampler(self.dataset, rank=rank, world_size=world)
        # num_workers is accepted but unused: the batch is produced by one device launch
        super().__init__(self.dataset, batch_size, shuffle=False, num_workers=0, collate_fn=self.dataset.collate,
                         sampler=sampler)

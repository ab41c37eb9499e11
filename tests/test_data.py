"""Data layer (CPU): IDX reader, MNIST loader, synthetic ImageNet loader sharding."""
import gzip
import struct

import numpy as np
import torch

from pytorch_distributed_template_amd.data import (EvalShardSampler, MnistDataLoader, SyntheticImageNetLoader,
                                                   read_idx, shard_bounds)


def _write_idx(path, arr, gz=False):
    code = {np.uint8: 0x08}[arr.dtype.type]
    hdr = bytes([0, 0, code, arr.ndim]) + b"".join(struct.pack(">I", d) for d in arr.shape)
    raw = hdr + arr.tobytes()
    path.write_bytes(gzip.compress(raw) if gz else raw)


def test_idx_reader_and_mnist_files(tmp_path):
    raw = tmp_path / "MNIST" / "raw"
    raw.mkdir(parents=True)
    imgs = np.random.RandomState(0).randint(0, 256, (20, 28, 28)).astype(np.uint8)
    lbls = (np.arange(20) % 10).astype(np.uint8)
    _write_idx(raw / "t10k-images-idx3-ubyte.gz", imgs, gz=True)
    _write_idx(raw / "t10k-labels-idx1-ubyte", lbls)
    assert (read_idx(raw / "t10k-images-idx3-ubyte.gz") == imgs).all()
    dl = MnistDataLoader(str(tmp_path), batch_size=8, shuffle=False, num_workers=0, training=False)
    assert dl.dataset.source.endswith("raw") and len(dl.dataset) == 20
    x, y = next(iter(dl))
    assert x.shape == (8, 1, 28, 28) and x.dtype == torch.float32
    ref = (torch.from_numpy(imgs[:8]).float() / 255 - 0.1307) / 0.3081
    assert torch.allclose(x[:, 0], ref, atol=1e-6) and y.tolist() == list(range(8))


def test_mnist_synthetic_fallback_is_deterministic():
    a = MnistDataLoader("/nonexistent", batch_size=4, shuffle=False, num_workers=0, training=True,
                        synthetic_size=32)
    b = MnistDataLoader("/nonexistent", batch_size=4, shuffle=False, num_workers=0, training=True,
                        synthetic_size=32)
    assert a.dataset.source == "synthetic" and len(a.dataset) == 32
    assert torch.equal(a.dataset.data, b.dataset.data)


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 37, 64):
        for w in (1, 2, 3, 8):
            idx = [i for r in range(w) for i in range(*shard_bounds(n, r, w))]
            assert idx == list(range(n))
    assert len(EvalShardSampler(10, rank=1, world_size=4)) == 3


def test_synthetic_imagenet_loader_cpu():
    dl = SyntheticImageNetLoader(batch_size=4, num_samples=10, pool=2, image_size=32, num_classes=5,
                                 training=False)
    batches = list(dl)
    assert len(dl) == 3 and [b[0].shape[0] for b in batches] == [4, 4, 2]
    x, y = batches[0]
    assert x.shape == (4, 3, 32, 32) and x.is_contiguous(memory_format=torch.channels_last)
    assert x.dtype == torch.float32 and -1 <= float(x.min()) and float(x.max()) < 1
    assert y.dtype == torch.int64 and int(y.max()) < 5
    assert len(dl.dataset) == 10
    tl = SyntheticImageNetLoader(batch_size=4, num_samples=10, pool=2, image_size=8, mode="pool")
    tl.set_epoch(1)
    assert torch.equal(next(iter(tl))[0], tl._pool[1][0])


def test_synthetic_imagenet_is_index_addressable_and_sampler_sharded():
    """The config loader is SyntheticImageNet -> DistributedSampler -> BaseDataLoader
    (/root/reference/data_loader/data_loaders.py:23-26): every index batch is
    materialised per sample index, ranks get disjoint shards, set_epoch reshuffles."""
    from torch.utils.data import DistributedSampler
    from pytorch_distributed_template_amd.base import BaseDataLoader
    dl = SyntheticImageNetLoader(batch_size=4, num_samples=10, image_size=8, num_classes=7)
    assert isinstance(dl, BaseDataLoader) and isinstance(dl.sampler, DistributedSampler)
    ds = dl.dataset
    order0 = list(iter(dl.sampler))
    x, y = next(iter(dl))
    for b, i in enumerate(order0[:4]):  # batch row b is sample order0[b]
        xi, yi = ds[i]
        assert torch.equal(x[b], xi) and int(y[b]) == int(yi)
    assert -1 <= float(x.min()) and float(x.max()) < 1 and 0 <= int(y.min()) and int(y.max()) < 7
    dl.set_epoch(1)
    assert list(iter(dl.sampler)) != order0 and sorted(iter(dl.sampler)) == sorted(order0)
    # two ranks: disjoint shards covering the (padded) dataset, equal step counts
    from pytorch_distributed_template_amd.data.synthetic import SyntheticImageNet
    shards = [list(DistributedSampler(ds, num_replicas=2, rank=r, shuffle=True, seed=0)) for r in range(2)]
    assert len(shards[0]) == len(shards[1]) == 5 and set(shards[0]) | set(shards[1]) == set(range(10))
    # same (seed, index) -> same sample, another seed -> another sample
    a, b = SyntheticImageNet(10, image_size=8, seed=3), SyntheticImageNet(10, image_size=8, seed=4)
    assert torch.equal(a[5][0], SyntheticImageNet(10, image_size=8, seed=3)[5][0]) and not torch.equal(a[5][0], b[5][0])

"""Samplers for one-process-per-GPU data parallelism.

Reference behaviour (``/root/reference/data_loader/data_loaders.py:23-26``):
a ``DistributedSampler`` for every split, never ``set_epoch``-ed,
which pads validation/test shards with duplicated samples.

Here:
  * training uses ``torch.utils.data.DistributedSampler`` (shuffled, padded so
    every rank runs the same number of steps -- DDP needs that) and the loader
    forwards ``set_epoch`` so each epoch reshuffles;
  * evaluation uses :class:`EvalShardSampler`: contiguous, *unpadded* shards
    whose union is exactly ``range(len(dataset))``, so gathered predictions
    contain no duplicates and metrics are over the true dataset.
"""
from __future__ import annotations

from torch.utils.data import Sampler


def shard_bounds(n: int, rank: int, world: int):
    """[start, stop) of rank's contiguous shard of ``n`` items (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


class EvalShardSampler(Sampler):
    def __init__(self, dataset_or_len, rank: int | None = None, world_size: int | None = None):
        from ..utils import dist as pdist
        n = dataset_or_len if isinstance(dataset_or_len, int) else len(dataset_or_len)
        self.rank = pdist.get_rank() if rank is None else rank
        self.world_size = pdist.get_world_size() if world_size is None else world_size
        self.start, self.stop = shard_bounds(n, self.rank, self.world_size)

    def __iter__(self):
        return iter(range(self.start, self.stop))

    def __len__(self):
        return self.stop - self.start

    def set_epoch(self, epoch: int):  # order is fixed; kept for a uniform loader API
        pass

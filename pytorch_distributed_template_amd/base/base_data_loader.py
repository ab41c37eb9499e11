"""BaseDataLoader (reference: ``/root/reference/base/base_data_loader.py:6-28``).

A ``DataLoader`` that, when given a sampler, forces ``shuffle=False`` and
passes the sampler through; otherwise shuffles itself. Stores
``init_kwargs`` like the reference. Adds ``set_epoch`` (forwarded to a
``DistributedSampler`` so each epoch reshuffles -- the reference never
called it) and ``n_samples`` for progress reporting.
"""
from torch.utils.data import DataLoader
from torch.utils.data.dataloader import default_collate


class BaseDataLoader(DataLoader):
    def __init__(self, dataset, batch_size, shuffle, num_workers, collate_fn=default_collate,
                 sampler=None, pin_memory=False, drop_last=False):
        self.init_kwargs = {
            "dataset": dataset,
            "batch_size": batch_size,
            "shuffle": False if sampler is not None else shuffle,
            "collate_fn": collate_fn,
            "num_workers": num_workers,
        }
        self.n_samples = len(sampler) if sampler is not None else len(dataset)
        extra = dict(pin_memory=pin_memory, drop_last=drop_last)
        if num_workers > 0:
            extra["persistent_workers"] = True
        if sampler is not None:
            super().__init__(sampler=sampler, **self.init_kwargs, **extra)
        else:
            super().__init__(**self.init_kwargs, **extra)

    def set_epoch(self, epoch: int):
        if hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

"""Misc utilities (reference: ``/root/reference/utils/util.py:9-67``).

Differences from the reference, all deliberate:
  * ``MetricTracker`` keeps its running sums in plain Python dicts instead of a
    pandas DataFrame (pandas is not a dependency; the reference's chained
    assignment warns on pandas 2.x and breaks under copy-on-write -- SURVEY
    §2.1 C15). Same API: ``reset/update/avg/result``.
  * ``MetricTracker.update`` accepts device tensors and defers the host sync
    until ``result()``/``avg()`` is called, so the training hot loop does not
    force a device->host sync every iteration.
"""
from __future__ import annotations

import json
from collections import OrderedDict
from itertools import repeat
from pathlib import Path

import torch


def set_deterministic(on: bool):
    """``--deterministic``: MIOpen/torch deterministic algorithms AND fixed native
    kernel variants (no autotune timing: the shipped table or the heuristic, the
    same on every run and rank; every reduction in csrc/ is atomic-free)."""
    if on:
        import os
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False
        os.environ["PDT_DETERMINISTIC"] = "1"


def seed_everything(seed, deterministic=False):
    """``--seed`` (reference train.py:101-106 / test.py:120-125, whose test.py seeds numpy
    without importing it): torch, numpy and Python RNGs, then ``set_deterministic``."""
    import random

    import numpy as np
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)
    torch.backends.cudnn.deterministic = deterministic
    torch.backends.cudnn.benchmark = False
    set_deterministic(deterministic)


def ensure_dir(dirname):
    dirname = Path(dirname)
    if not dirname.is_dir():
        dirname.mkdir(parents=True, exist_ok=True)


def read_json(fname):
    fname = Path(fname)
    with fname.open("rt") as handle:
        return json.load(handle, object_hook=OrderedDict)


def write_json(content, fname):
    fname = Path(fname)
    with fname.open("wt") as handle:
        json.dump(content, handle, indent=4, sort_keys=False)


def inf_loop(data_loader):
    """Wrapper for an endless data loader (iteration-based training)."""
    for loader in repeat(data_loader):
        yield from loader


class MetricTracker:
    """Running weighted averages per key.

    ``update(key, value, n)`` accepts python numbers or 0-d tensors (kept on
    their device and summed lazily).
    """

    def __init__(self, *keys, writer=None):
        self.writer = writer
        self._keys = list(keys)
        self.reset()

    def reset(self):
        self._total = {k: 0.0 for k in self._keys}
        self._counts = {k: 0 for k in self._keys}
        self._pending = {k: [] for k in self._keys}

    def _ensure(self, key):
        if key not in self._total:
            self._keys.append(key)
            self._total[key] = 0.0
            self._counts[key] = 0
            self._pending[key] = []

    def update(self, key, value, n=1, write=True):
        self._ensure(key)
        if self.writer is not None and write:
            self.writer.add_scalar(key, value)
        if isinstance(value, torch.Tensor):
            self._pending[key].append(value.detach().float() * n)
        else:
            self._total[key] += float(value) * n
        self._counts[key] += n

    def _flush(self, key):
        pend = self._pending[key]
        if pend:
            self._total[key] += float(torch.stack([p.reshape(()) for p in pend]).sum().item())
            self._pending[key] = []

    def avg(self, key):
        self._flush(key)
        c = self._counts[key]
        return self._total[key] / c if c else 0.0

    def result(self):
        return {k: self.avg(k) for k in self._keys}

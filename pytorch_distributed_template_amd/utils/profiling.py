"""Lightweight step-phase profiling (the reference has none -- SURVEY §5).

``PhaseTimer`` brackets named phases of a training step (forward, backward,
optimizer, ...) with HIP events on the current stream and reports mean device
milliseconds per phase without forcing a host sync inside the step: events
are resolved lazily in ``summary()``. Each phase is also a ROCTx range
(``torch.cuda.nvtx`` maps to roctx on ROCm), so ``rocprofv3 --marker-trace``
timelines show the phases.

    timer = PhaseTimer(enabled=True)
    with timer.phase("forward"):
        out = model(x)
    ...
    timer.summary()  # {"forward": 9.1, "backward": 17.9, "optimizer": 0.3}
"""
from __future__ import annotations

import contextlib
from collections import defaultdict

import torch


class PhaseTimer:
    def __init__(self, enabled: bool = True, max_pending: int = 4096):
        self.enabled = enabled and torch.cuda.is_available()
        self._pending = []
        self._tot = defaultdict(float)
        self._cnt = defaultdict(int)
        self._max_pending = max_pending

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.nvtx.range_push(name)
        e0.record()
        try:
            yield
        finally:
            e1.record()
            torch.cuda.nvtx.range_pop()
            self._pending.append((name, e0, e1))
            if len(self._pending) > self._max_pending:
                self._resolve()

    def _resolve(self):
        for name, e0, e1 in self._pending:
            e1.synchronize()
            self._tot[name] += e0.elapsed_time(e1)
            self._cnt[name] += 1
        self._pending.clear()

    def summary(self, reset: bool = True):
        self._resolve()
        out = {k: self._tot[k] / max(self._cnt[k], 1) for k in self._tot}
        if reset:
            self._tot.clear()
            self._cnt.clear()
        return out

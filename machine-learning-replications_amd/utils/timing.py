"""Stage timers (device-synchronised wall clock) + optional roctx ranges.

The reference has no timing at all (``from time import time`` is imported but
unused, ``train_ensemble_public.py:6``); this gives per-stage tables for the
bench and JSON-lines run logs.
"""
from __future__ import annotations

import contextlib
import json
import time
from collections import OrderedDict

import torch

try:  # roctx ranges show up in rocprofv3 --marker-trace
    from torch.cuda import nvtx as _nvtx  # PyTorch routes this to roctx on ROCm
except Exception:  # pragma: no cover
    _nvtx = None


class StageTimer:
    def __init__(self, enabled: bool = True, sync: bool = True, device=None):
        self.enabled = enabled
        self.sync = sync
        self.device = device
        self.times = OrderedDict()

    def _sync(self):
        if self.sync and torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize(self.device)

    @contextlib.contextmanager
    def stage(self, name: str):
        if not self.enabled:
            yield
            return
        self._sync()
        if _nvtx is not None and torch.cuda.is_available():
            try:
                _nvtx.range_push(name)
            except Exception:
                pass
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self._sync()
            dt = time.perf_counter() - t0
            if _nvtx is not None and torch.cuda.is_available():
                try:
                    _nvtx.range_pop()
                except Exception:
                    pass
            self.times[name] = self.times.get(name, 0.0) + dt

    def total(self) -> float:
        return sum(self.times.values())

    def table(self) -> str:
        w = max([len(k) for k in self.times] + [5])
        lines = [f"{'stage':<{w}}  seconds"]
        for k, v in self.times.items():
            lines.append(f"{k:<{w}}  {v:8.4f}")
        lines.append(f"{'total':<{w}}  {self.total():8.4f}")
        return "\n".join(lines)

    def json(self) -> str:
        return json.dumps({k: round(v, 6) for k, v in self.times.items()})

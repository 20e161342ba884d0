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
    """``sync=True``: device-synchronised wall clock per stage.  ``events=True``: no host
    synchronisation at all — a timing event pair on the current stream per stage (stages end by
    joining their side streams into it) plus the host-side wall time of the stage's Python; read
    both with :meth:`collect` after the caller's own synchronisation.  The bench uses the event
    form inside its timed steps, so the per-stage table costs the timed region nothing."""

    def __init__(self, enabled: bool = True, sync: bool = True, device=None, events: bool = False):
        self.enabled = enabled
        self.events = events and torch.cuda.is_available()
        self.sync = sync and not self.events
        self.device = device
        self.times = OrderedDict()
        self.host_times = OrderedDict()
        self._pending = []

    def _sync(self):
        if self.sync and torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize(self.device)

    @contextlib.contextmanager
    def stage(self, name: str):
        if not self.enabled:
            yield
            return
        if self.events:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            h0 = time.perf_counter()
            try:
                yield
            finally:
                e1.record()
                self.host_times[name] = self.host_times.get(name, 0.0) + time.perf_counter() - h0
                self._pending.append((name, e0, e1))
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

    def collect(self) -> "StageTimer":
        """Resolve pending event pairs into ``times`` (device timeline, seconds); the events
        must be complete (call after a synchronisation)."""
        for name, e0, e1 in self._pending:
            self.times[name] = self.times.get(name, 0.0) + e0.elapsed_time(e1) * 1e-3
        self._pending = []
        return self

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


# ---------------------------------------------------------------------------- host timeline marks
# HFENS_TRACE_HOST=1: ``hmark(name)`` records host wall-clock points anywhere in the fit; the
# stacking trainer prints them per fit (ms since the first mark).  Zero cost when disabled.
import os as _os

TRACE_HOST = _os.environ.get("HFENS_TRACE_HOST", "0") == "1"
_MARKS: list = []


def hmark(name: str) -> None:
    if TRACE_HOST:
        _MARKS.append((name, time.perf_counter()))


def _rank_prefix(prefix: str) -> str:
    """"[host]" → "[host r1]" on rank 1 of a multi-process run (torchrun: the ranks share stderr)."""
    if int(_os.environ.get("WORLD_SIZE", "1")) > 1:
        return prefix[:-1] + f" r{_os.environ.get('RANK', '0')}]"
    return prefix


def hmarks_flush(prefix: str = "[host]") -> None:
    if TRACE_HOST and _MARKS:
        import sys
        prefix = _rank_prefix(prefix)
        t0 = _MARKS[0][1]
        print(prefix + " " + " ".join(f"{k}={1e3 * (v - t0):.2f}" for k, v in _MARKS), file=sys.stderr)
        _MARKS.clear()


# ---------------------------------------------------------------------------- device timeline marks
# HFENS_TRACE_DEV=1: ``dmark(name)`` records a timing event on the current stream; ``dmarks_flush``
# (end of ``pipeline.develop``) prints when the device reached each one, in ms since the first mark
# (recorded at develop() entry on an idle device, so the numbers line up with the host marks).
# Diagnostic only: no profiler attached, so the streams overlap as in a normal run.
TRACE_DEV = _os.environ.get("HFENS_TRACE_DEV", "0") == "1"
_DMARKS: list = []


def dmark(name: str) -> None:
    if TRACE_DEV:
        import torch
        if torch.cuda.is_available():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _DMARKS.append((name, e))


def dmarks_flush(prefix: str = "[dev]") -> None:
    if TRACE_DEV and _DMARKS:
        import sys
        prefix = _rank_prefix(prefix)
        for _, e in _DMARKS:
            e.synchronize()
        e0 = _DMARKS[0][1]
        print(prefix + " " + " ".join(f"{k}={e0.elapsed_time(e):.2f}" for k, e in _DMARKS), file=sys.stderr)
        _DMARKS.clear()

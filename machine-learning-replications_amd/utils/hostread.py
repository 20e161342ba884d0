"""Early host read-backs that do not wait on their events.

A small device result needed on the host (a selection, the SMO's early read, the Platt pairs, error
words and input guards) is copied into pinned memory right behind the kernel that produces it, with
an event.  On this ROCm stack those events reported completion late — when work enqueued behind
them had drained (up to ≈ 1 ms in the stacking fit's tail, ``profiles/r6_runs/r6aq``) — although
the data itself had landed.  :func:`stage` therefore pre-fills the pinned buffer with a sentinel no
producer writes (NaN for floating point, :data:`SENTINEL` for integers) and :func:`landed` polls
the buffer until no sentinel remains, falling back to the event after ``budget_s`` (a value that
really is the sentinel, or a slow copy)."""
from __future__ import annotations

import time

import numpy as np
import torch

SENTINEL = -0x5EED5EED       # integer fill: no error word, flag or index equals it


def stage(dev: torch.Tensor, stream=None):
    """(pinned host copy, event) of ``dev``, enqueued on ``stream`` (default: the current one).
    Booleans travel as int32 (a bool buffer has no sentinel value)."""
    if dev.dtype == torch.bool:
        dev = dev.to(torch.int32)
    host = torch.empty(dev.shape, dtype=dev.dtype, pin_memory=True)
    host.fill_(float("nan") if dev.dtype.is_floating_point else SENTINEL)
    host.copy_(dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(stream) if stream is not None else ev.record()
    return host, ev


def _pending(a: np.ndarray) -> bool:
    if a.dtype.kind == "f":
        return bool(np.isnan(a).any())
    return bool((a == SENTINEL).any())


def landed(host: torch.Tensor, ev, budget_s: float = 0.05) -> np.ndarray:
    """``host`` as a numpy array once every element has been written (see the module docstring)."""
    a = host.numpy()
    t_end = time.perf_counter() + budget_s
    while _pending(a):
        if time.perf_counter() > t_end:
            ev.synchronize()
            break
    return a

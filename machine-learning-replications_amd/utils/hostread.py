"""Early host read-backs that do not wait on their events.

A small device result needed on the host (a selection, the SMO's early read, the Platt pairs, error
words and input guards) is copied into pinned memory right behind the kernel that produces it, with
an event.  On this ROCm stack those events reported completion late — when work enqueued behind
them had drained (up to ≈ 1 ms in the stacking fit's tail, ``profiles/r6_runs/r6aq``) — although
the data itself had landed.  :func:`stage` therefore pre-fills the pinned buffer with a sentinel no
producer writes (NaN for floating point, :data:`SENTINEL` for integers) and :func:`landed` polls
the buffer until no sentinel remains, falling back to the event after ``budget_s`` (a value that
really is the sentinel, or a slow copy).

With :data:`KERNEL_STORE` the words leave the device as system-scope stores from a small kernel on
the producer's own queue (``ops/csrc/hostread.hip host_store``) instead of an async copy, whose
copy engine first has to observe the compute queue's kernel finish.  Torch's pinned allocator does
not know that kernel writes the buffer, so the buffer is kept referenced here until its event has
completed (:data:`_INFLIGHT`): a read a caller abandons cannot land in a recycled block."""
from __future__ import annotations

import os
import time

import numpy as np
import torch

SENTINEL = -0x5EED5EED       # integer fill: no error word, flag or index equals it


KERNEL_STORE = os.environ.get("HFENS_HOSTREAD_KERNEL", "0") != "0"   # (measured neutral: r6bq)
_INFLIGHT: list = []      # (host buffer, event) of kernel-written reads not yet known complete


def _kernel_store(dev: torch.Tensor, host: torch.Tensor) -> bool:
    if not (KERNEL_STORE and dev.is_cuda and dev.element_size() in (4, 8) and dev.is_contiguous()):
        return False
    from .. import ops
    E = ops.ext()
    if E is None or not hasattr(E, "host_store"):
        return False
    E.host_store(dev.data_ptr(), host.data_ptr(), int(dev.numel()), int(dev.element_size()),
                 torch.cuda.current_stream(dev.device).cuda_stream)
    return True


def stage(dev: torch.Tensor, stream=None):
    """(pinned host copy, event) of ``dev``, enqueued on the current stream (``stream``: where the
    event is recorded; default the current one).  Booleans travel as int32 (a bool buffer has no
    sentinel value)."""
    if dev.dtype == torch.bool:
        dev = dev.to(torch.int32)
    host = torch.empty(dev.shape, dtype=dev.dtype, pin_memory=True)
    host.fill_(float("nan") if dev.dtype.is_floating_point else SENTINEL)
    kern = _kernel_store(dev, host)
    if not kern:
        host.copy_(dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(stream) if stream is not None else ev.record()
    if kern:
        _INFLIGHT[:] = [(h, e) for h, e in _INFLIGHT if not e.query()]
        _INFLIGHT.append((host, ev))
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

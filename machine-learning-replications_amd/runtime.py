"""Device runtime helpers: persistent HIP streams and persistent workspaces.

Why this exists (measured, ``profiles/r2_driver_gap.md``): the concurrent base-model fit used
to create fresh ``torch.cuda.Stream`` objects every fit.  PyTorch hands those out round-robin
from a pool, and its caching allocator keys cached blocks by stream, so the 7 GB batched SVM
Gram allocated on "the" side stream was a NEW block almost every fit.  Cached blocks piled up
on ~30 pool streams until HBM was full, then the allocator synchronised and released
everything — a 0.3–2 s stall every few fits (the driver's 285 ms/fit mean over a 88 ms median).

Here every role gets ONE stream per device for the life of the process, and the big per-fit
buffers (Gram matrices, SMO exchange slots) are process-lifetime workspaces that only grow.
A workspace remembers the stream that last used it; handing it to another stream makes that
stream wait for everything already enqueued on the previous one.
"""
from __future__ import annotations

from typing import Dict, Tuple

import threading

import os

import torch

_STREAMS: Dict[Tuple[torch.device, str], torch.cuda.Stream] = {}
_WS: Dict[Tuple[torch.device, str], list] = {}


def stream(device, role: str, priority: int = 0) -> "torch.cuda.Stream":
    """The process-lifetime stream for ``role`` on ``device`` (created on first use)."""
    d = torch.device(device)
    key = (d, role)
    s = _STREAMS.get(key)
    if s is None:
        s = torch.cuda.Stream(d, priority=priority)
        _STREAMS[key] = s
    return s


# The development fit's streams in ONE creation order.  HIP multiplexes streams onto a few hardware
# queues per priority level as they are created (GPU_MAX_HW_QUEUES), so which streams share a
# queue — i.e. which kernels serialise behind each other — depends on the order of first use.
# Measured (profiles/r5_headline.md): enqueuing the SVC batch earlier changed that order and cost
# the SMO 3-5 ms; creating every role here first keeps the measured-good assignment whatever the
# code path.
# (svc_ws_1, the 8k-point problems' working-set group, at normal priority: the critical group's
# launches then dispatch ahead of its — measured 16.4 / 16.7 vs 17.1 / 17.0 ms per fit on one box,
# profiles/r6_runs/r6az; svc_ws_2: the smallest group's own stream when smo.WS_LAST_SIDE)
FIT_STREAMS = (("aux", 0), ("lasso_refit", 0), ("svc", int(os.environ.get("HFENS_SVC_PRIORITY", "-1"))), ("bases", 0),
               ("svc_ws_0", -1),
               ("svc_ws_1", int(os.environ.get("HFENS_WS1_PRIORITY", "0"))))
if os.environ.get("HFENS_SVM_WS_LAST_SIDE", "0") == "1" and os.environ.get("HFENS_SVM_WS_GROUPS", "3") != "2":
    # (measured slower at either priority: the extra stream shared a hardware queue with the GBC /
    # LassoCV streams, or slowed the SMO — profiles/r6_runs/r6ba, r6bb)
    FIT_STREAMS += (("svc_ws_2", int(os.environ.get("HFENS_WS2_PRIORITY", "0"))),)


def init_fit_streams(device) -> None:
    d = torch.device(device)
    if d.type != "cuda" or (d, FIT_STREAMS[-1][0]) in _STREAMS:
        return
    for role, prio in FIT_STREAMS:
        stream(d, role, priority=prio)


def workspace(device, name: str, numel: int, dtype=torch.float32) -> torch.Tensor:
    """A ``numel``-element view of a process-lifetime buffer (grown, never shrunk).

    Contents are undefined.  Ordering: the caller's current stream is made to wait for the work
    already enqueued on the stream that last took this workspace (host program order means every
    earlier user's kernels are enqueued by now)."""
    d = torch.device(device)
    key = (d, name)
    ent = _WS.get(key)
    nbytes = int(numel) * torch.empty(0, dtype=dtype).element_size()
    cur = torch.cuda.current_stream(d) if d.type == "cuda" else None
    if ent is not None and cur is not None and ent[1] is not None and ent[1] != cur:
        ev = torch.cuda.Event()
        ev.record(ent[1])
        cur.wait_event(ev)
    if ent is None or ent[0].numel() < nbytes:
        if ent is not None:
            ent[0] = None          # drop the old buffer first: peak = one copy (record_stream
            #                        below keeps the allocator from recycling it under live work)
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=d)
        ent = [buf, cur]
        _WS[key] = ent
    elif cur is not None and ent[1] != cur:
        ent[0].record_stream(cur)
    ent[1] = cur
    return ent[0][:nbytes].view(dtype)[:numel]


def release_workspaces(device=None):
    """Free every workspace (of ``device``, or all)."""
    for key in list(_WS):
        if device is None or key[0] == torch.device(device):
            del _WS[key]


_PINNED = threading.local()


def host_read(t: torch.Tensor) -> torch.Tensor:
    """``t.cpu()`` for a small device tensor WITHOUT a spinning host thread: a non-blocking copy
    into a per-thread pinned buffer, then a wait on a blocking-sync event (hipEventBlockingSync:
    the thread sleeps in the driver instead of polling).  The interior-point solves read their
    convergence state once per iteration from 4 host threads; spinning reads made the 1M-row fit
    use ~2.9 CPU-seconds per second.  Returns a host tensor the caller may keep."""
    if not t.is_cuda:
        return t
    t = t.contiguous()
    key = (t.device, t.dtype)
    bufs = getattr(_PINNED, "bufs", None)
    if bufs is None:
        bufs = _PINNED.bufs = {}
    buf = bufs.get(key)
    if buf is None or buf.numel() < t.numel():
        buf = bufs[key] = torch.empty(max(64, t.numel()), dtype=t.dtype, pin_memory=True)
    out = buf[: t.numel()]
    out.copy_(t.reshape(-1), non_blocking=True)
    ev = torch.cuda.Event(blocking=True)
    ev.record(torch.cuda.current_stream(t.device))
    ev.synchronize()
    return out.reshape(t.shape).clone()


def blocking_sync(enable: bool = True) -> bool:
    """hipSetDeviceFlags(hipDeviceScheduleBlockingSync) on the current device BEFORE torch creates
    its context: every host wait (stream / event synchronisation, blocking copies) then sleeps on
    the completion signal instead of spinning a core.  For long device-bound runs (config 3: four
    interior-point threads that each wait once per iteration); latency-bound fits keep the default
    spin (a sleeping waiter wakes tens of µs late).  Returns whether the flag was set."""
    if not enable:
        return False
    import ctypes
    import os
    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    try:
        hip = ctypes.CDLL(lib if os.path.exists(lib) else "libamdhip64.so")
        return hip.hipSetDeviceFlags(ctypes.c_uint(0x4)) == 0   # hipDeviceScheduleBlockingSync
    except OSError:
        return False

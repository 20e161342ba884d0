"""Which of the development fit's streams share a hardware queue (HIP maps streams onto
GPU_MAX_HW_QUEUES queues as they are created; kernels of streams on one queue serialise).

For every ordered pair (A, B) of the fit's streams, created in runtime.FIT_STREAMS order plus the
roles created later: a ~4 ms spin kernel on A, then a tiny kernel on B; B's completion time shows
whether B waited behind A (shared queue) or ran at once.  Prints the sharing matrix."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from hfens import runtime  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
runtime.init_fit_streams(dev)
extra = [r.split(":") for r in os.environ.get("HWQ_EXTRA", "lasso_spec:-1,lasso_path:0").split(",") if r]
for role, prio in extra:
    runtime.stream(dev, role, priority=int(prio))
roles = [r for r, _ in runtime.FIT_STREAMS] + [r for r, _ in extra]
streams = {r: runtime.stream(dev, r) for r in roles}
streams["main"] = torch.cuda.current_stream(dev)
roles = ["main"] + roles
x = torch.zeros(16, device=dev)
torch.cuda._sleep(1000)
torch.cuda.synchronize()
# calibrate the spin: cycles for ~4 ms
c = 1 << 22
for _ in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(c)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    c = int(c * 4.0 / max(ms, 1e-3))
print(f"spin cycles {c} ≈ 4 ms", flush=True)
shared = {}
for a in roles:
    for b in roles:
        if a == b:
            continue
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        tb = torch.cuda.Event(enable_timing=True)
        ta = torch.cuda.Event(enable_timing=True)
        t0.record(streams[a])
        with torch.cuda.stream(streams[a]):
            torch.cuda._sleep(c)
        ta.record(streams[a])
        time.sleep(0.0005)     # (A's packets reach its queue first)
        with torch.cuda.stream(streams[b]):
            x.add_(1.0)
        tb.record(streams[b])
        torch.cuda.synchronize()
        shared[(a, b)] = t0.elapsed_time(tb) > 0.6 * t0.elapsed_time(ta)
w = max(len(r) for r in roles)
print(" " * (w + 1) + " ".join(r[:6].rjust(6) for r in roles))
for a in roles:
    print(a.ljust(w) + " " + " ".join(("  --  " if a == b else ("  XX  " if shared[(a, b)] else "   .  ")) for b in roles))
print("XX: a tiny kernel on the column's stream waited behind a 4 ms kernel on the row's stream")

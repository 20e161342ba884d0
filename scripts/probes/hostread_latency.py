"""Latency of a small device→host read-back: async pinned copy vs the host_store kernel
(ops/csrc/hostread.hip), each staged right behind a ~0.1 ms producer kernel on an otherwise idle
stream.  Prints the median host time from enqueue to landed() per method (lower = the read lands
sooner after its producer).  Usage: python scripts/probes/hostread_latency.py [REPS]"""
import sys
import time
from statistics import median

import torch

sys.path.insert(0, ".")
from hfens.utils import hostread  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
a = torch.randn(2048, 2048, device="cuda")
small = torch.zeros(16, dtype=torch.float64, device="cuda")
res = {}
for rnd in range(2):
    for kernel in (False, True):
        hostread.KERNEL_STORE = kernel
        ts = []
        for i in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b = a @ a                       # the producer's predecessor (~0.1 ms)
            v = small + b[0, :16].to(torch.float64)
            host, ev = hostread.stage(v)
            hostread.landed(host, ev, budget_s=1.0)
            ts.append(time.perf_counter() - t0)
        res.setdefault(kernel, []).append(median(ts[20:]) * 1e3)
torch.cuda.synchronize()
ref = []
for i in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b = a @ a
    v = small + b[0, :16].to(torch.float64)
    torch.cuda.synchronize()
    ref.append(time.perf_counter() - t0)
print(f"hostread latency medians (ms, enqueue→landed): copy {res[False]} kernel {res[True]} "
      f"(producer chain + synchronize: {median(ref[20:]) * 1e3:.3f})")

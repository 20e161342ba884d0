"""The interior point's r × r factor and solves (linalg.hip chol_spd_mw / chol_solve, r = 428) alone,
beside a stream of large f64 GEMMs (the other problems' weighted Grams), and on a high-priority
stream beside the same GEMMs: per-factor+3-solve latency."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens import ops  # noqa: E402

E = ops.ext()
dev = torch.device("cuda")
r = 428
A = torch.randn(4 * r, r, dtype=torch.float64, device=dev)
S = A.T @ A + torch.eye(r, dtype=torch.float64, device=dev)
Lc = torch.empty(r, r, dtype=torch.float64, device=dev)
scv = torch.empty(r, dtype=torch.float64, device=dev)
info = torch.zeros(1, dtype=torch.int32, device=dev)
chw = torch.zeros(4, dtype=torch.int32, device=dev)
chpt = torch.empty(32 * r, dtype=torch.float64, device=dev)
B2 = torch.randn(r, 2, dtype=torch.float64, device=dev)
B1 = torch.randn(r, 1, dtype=torch.float64, device=dev)
P = torch.randn(8, 8192, r, dtype=torch.float64, device=dev)


def chain(st):
    sp = st.cuda_stream
    E.chol_spd_mw(S.data_ptr(), r, Lc.data_ptr(), scv.data_ptr(), info.data_ptr(), chw.data_ptr(), chpt.data_ptr(), sp)
    E.chol_solve(Lc.data_ptr(), scv.data_ptr(), r, 2, B2.data_ptr(), sp)
    E.chol_solve(Lc.data_ptr(), scv.data_ptr(), r, 1, B1.data_ptr(), sp)
    E.chol_solve(Lc.data_ptr(), scv.data_ptr(), r, 1, B1.data_ptr(), sp)


def timed(st, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n):
        chain(st)
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / n


lo = torch.cuda.Stream()
hi = torch.cuda.Stream(priority=-1)
bg = [torch.cuda.Stream() for _ in range(3)]
for _ in range(3):
    timed(lo, 2)
torch.cuda.synchronize()
print(f"alone: {timed(lo):.3f} ms per factor + 3 solves", flush=True)
for name, st in (("normal", lo), ("high-priority", hi)):
    torch.cuda.synchronize()
    for b in bg:
        with torch.cuda.stream(b):
            for _ in range(40):
                torch.bmm(P.transpose(1, 2), P)
    ms = timed(st)
    torch.cuda.synchronize()
    print(f"beside 3 GEMM streams, {name}: {ms:.3f} ms", flush=True)
t0 = time.perf_counter()
for b in bg:
    with torch.cuda.stream(b):
        for _ in range(10):
            torch.bmm(P.transpose(1, 2), P)
torch.cuda.synchronize()
print(f"GEMM batch alone: {(time.perf_counter() - t0) * 1e3 / 30:.3f} ms per bmm", flush=True)

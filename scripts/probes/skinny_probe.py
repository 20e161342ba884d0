"""Launch-shape sweep of the interior point's skinny passes over the f32 copy of Φ (1M × 428):
Φᵀ V (phit_f32) and Φ W (phi_gemv_f32), k = 1 and 2.  HFENS_PHIT_CFG / HFENS_GEMV_CFG =
"rows in flight, grid" (lowrank.hip skinny_cfg) are read per launch:
- phit "R,0" = the flat kernel (default "4,0"), "R,w" = the row-slab kernel at w workgroups/CU;
- gemv "R,3" = a wave per row with contiguous 1 KB loads (default "2,3"), "R,0" / "R,1" = a wave
  per row with 8-column lanes (8 or the resident workgroups per CU).
Prints µs per call, the HBM read rate of Φ and the difference from the default shape's result
(first in each list).  Records: profiles/r3_runs/skinny_probe.log."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens import ops  # noqa: E402

E = ops.ext()
dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
r = 428
g = torch.Generator(device=dev).manual_seed(3)
P = torch.randn(n, r, generator=g, device=dev, dtype=torch.float32)
st = ops.stream_ptr(dev)
GB = n * r * 4 / 1e9


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for k in (1, 2):
    V = torch.randn(n, k, generator=g, device=dev, dtype=torch.float64)
    W = torch.randn(r, k, generator=g, device=dev, dtype=torch.float64)
    ref = {}
    for cfg in ("4,0", "4,4", "2,0", "8,0", "4,7"):
        os.environ["HFENS_PHIT_CFG"] = cfg
        pl = torch.zeros(1, dtype=torch.int64)
        E.phit_part_len(n, r, k, pl.data_ptr())
        part = torch.empty(int(pl), dtype=torch.float64, device=dev)
        out = torch.empty(r, k, dtype=torch.float64, device=dev)
        us = timeit(lambda: E.phit_f32(P.data_ptr(), V.data_ptr(), n, r, k, part.data_ptr(), int(pl), out.data_ptr(), st))
        ref.setdefault("phit", out.clone())
        d = float((out - ref["phit"]).abs().max() / ref["phit"].abs().max())
        print(f"phit k={k} cfg {cfg}: {us:8.1f} us  {GB / us * 1e6 / 1e3:5.2f} TB/s  rel diff {d:.1e}", flush=True)
    os.environ.pop("HFENS_PHIT_CFG")
    for cfg in ("2,3", "4,0", "2,1", "4,3"):
        os.environ["HFENS_GEMV_CFG"] = cfg
        Y = torch.empty(n, k, dtype=torch.float64, device=dev)
        us = timeit(lambda: E.phi_gemv_f32(P.data_ptr(), W.data_ptr(), n, r, k, Y.data_ptr(), st))
        ref.setdefault("gemv", Y.clone())
        print(f"gemv k={k} cfg {cfg}: {us:8.1f} us  {GB / us * 1e6 / 1e3:5.2f} TB/s  equal {bool(torch.equal(Y, ref['gemv']))}",
              flush=True)
    os.environ.pop("HFENS_GEMV_CFG")

# reference streams: torch's sum (read only) and clone (read + write) of the same bytes
us = timeit(lambda: P.sum())
print(f"torch sum   : {us:8.1f} us  {GB / us * 1e6 / 1e3:5.2f} TB/s (read)", flush=True)
us = timeit(lambda: P.clone())
print(f"torch clone : {us:8.1f} us  {2 * GB / us * 1e6 / 1e3:5.2f} TB/s (read + write)", flush=True)
Pd = torch.empty(n, r, dtype=torch.float64, device=dev)
d = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
us = timeit(lambda: E.scale_rows_f32(P.data_ptr(), d.data_ptr(), n, r, Pd.data_ptr(), st))
print(f"scale_rows  : {us:8.1f} us  {3 * GB / us * 1e6 / 1e3:5.2f} TB/s (read f32 + write f64)", flush=True)

# the r × r factor and solves of the same iteration (linalg.hip chol_spd / chol_solve, one workgroup)
A = torch.randn(4 * r, r, generator=g, device=dev, dtype=torch.float64)
S = A.T @ A + torch.eye(r, device=dev, dtype=torch.float64)
Lc = torch.empty(r, r, dtype=torch.float64, device=dev)
scv = torch.empty(r, dtype=torch.float64, device=dev)
info = torch.zeros(1, dtype=torch.int32, device=dev)
us = timeit(lambda: E.chol_spd(S.data_ptr(), r, Lc.data_ptr(), scv.data_ptr(), info.data_ptr(), st))
print(f"chol_spd r={r}: {us:8.1f} us", flush=True)
for k in (1, 2):
    B0 = torch.randn(r, k, generator=g, device=dev, dtype=torch.float64)
    Bk = B0.clone()
    us = timeit(lambda: E.chol_solve(Lc.data_ptr(), scv.data_ptr(), r, k, Bk.data_ptr(), st))
    Bk.copy_(B0)
    E.chol_solve(Lc.data_ptr(), scv.data_ptr(), r, k, Bk.data_ptr(), st)
    res = float((S @ Bk - B0).abs().max() / B0.abs().max())
    print(f"chol_solve r={r} k={k}: {us:8.1f} us  residual {res:.1e}", flush=True)

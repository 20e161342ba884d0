"""Time the pieces of the low-rank SVC interior-point solver on one device (per-iteration cost).
python scripts/ipm_probe.py ROWS [LANDMARKS]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.models.svc_lowrank import _weighted_gram, ipm_svc_dual, nystrom_map  # noqa: E402


def tm(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / reps


def main():
    n = int(sys.argv[1])
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    Z = torch.randn(n, 17, generator=g, device=dev, dtype=torch.float64)
    y = torch.where(torch.rand(n, generator=g, device=dev) < 0.2, -1.0, 1.0).to(torch.float64)
    idx = torch.randperm(n, device=dev)[:m]
    t0 = time.perf_counter()
    Phi, T = nystrom_map(Z, idx, 1 / 17)
    torch.cuda.synchronize()
    print(f"rows {n} landmarks {m}: nystrom map {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    only_ipm = len(sys.argv) > 3 and sys.argv[3] == "ipm-only"
    d = torch.rand(n, device=dev, dtype=torch.float64)
    if only_ipm:
        c = torch.where(y > 0, 0.625, 2.5).to(torch.float64)
        # f64 Φ (skinny passes over f64) and Φ rounded to f32 (skinny passes over the f32 copy)
        maps = (("f64 map", Phi), ("f32-rounded map", Phi.to(torch.float32).to(torch.float64)))
        if len(sys.argv) > 4 and sys.argv[4] == "f32-only":
            maps = maps[1:]
        for tag, P in maps:
            ipm_svc_dual(P, y, c, max_iter=3)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a, rho, it = ipm_svc_dual(P, y, c)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"  ipm solve [{tag}] {1e3 * dt:.1f} ms, {it} iterations ({1e3 * dt / it:.2f} ms/iter), "
                  f"rho {rho:.6f}, sum(a) {float(a.sum()):.6f}", flush=True)
        return
    print(f"  weighted gram (split-K) {tm(lambda: _weighted_gram(Phi, d)):.2f} ms", flush=True)
    print(f"  weighted gram (one GEMM) {tm(lambda: Phi.T @ (d[:, None] * Phi)):.2f} ms", flush=True)
    S = torch.eye(Phi.shape[1], device=dev, dtype=torch.float64) + _weighted_gram(Phi, d)
    print(f"  cholesky {tm(lambda: torch.linalg.cholesky_ex(S)):.2f} ms", flush=True)
    v = torch.rand(n, 2, device=dev, dtype=torch.float64)
    from hfens.models.svc_lowrank import _phit
    print(f"  Phi^T v split-K {tm(lambda: _phit(Phi, v)):.2f} ms")
    print(f"  Phi^T v (2 rhs) {tm(lambda: Phi.T @ v):.2f} ms   Phi w {tm(lambda: Phi @ T[:, :2]):.2f} ms", flush=True)
    c = torch.where(y > 0, 0.625, 2.5).to(torch.float64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a, rho, it = ipm_svc_dual(Phi, y, c)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"  ipm solve {1e3 * dt:.1f} ms, {it} iterations ({1e3 * dt / it:.2f} ms/iter), rho {rho:.4f}", flush=True)


if __name__ == "__main__":
    main()

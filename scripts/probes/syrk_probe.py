"""Φᵀ diag(d) Φ at config-3 size (1M × 428 f64): the library split-K path with the full product
and with block-upper products of several block sizes (HFENS_SYRK_BLOCK), and the native kernel.
python scripts/probes/syrk_probe.py [ROWS] [RANK]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.models import svc_lowrank as sl  # noqa: E402


def tm(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    r = int(sys.argv[2]) if len(sys.argv) > 2 else 428
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    Phi = torch.randn(n, r, generator=g, device=dev, dtype=torch.float64).to(torch.float32).to(torch.float64)
    d = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 1e3
    sl.SYRK_BLOCK = 0
    ref = sl._weighted_gram(Phi, d)
    flops = 2.0 * n * r * r
    for bs in (0, 64, 96, 128, 160, 214):
        sl.SYRK_BLOCK = bs
        S = sl._weighted_gram(Phi, d)
        err = float(((S - ref).abs() / ref.abs().max()).max())
        t = tm(lambda: sl._weighted_gram(Phi, d))
        print(f"block {bs:4d}: {t:7.2f} ms  ({flops / t / 1e9:6.1f} full-product TF/s)  max rel diff {err:.2e}", flush=True)
    sl.SYRK_BLOCK = 0
    sl.NATIVE_SYRK = True
    S = sl._weighted_gram(Phi, d)
    err = float(((S - ref).abs() / ref.abs().max()).max())
    print(f"native wsyrk: {tm(lambda: sl._weighted_gram(Phi, d)):7.2f} ms  max rel diff {err:.2e}", flush=True)


if __name__ == "__main__":
    main()

"""Interior-point iterations vs the starting point (α₀ = A0·C, ν₀ = μ₀ = NU0) on a config-3-shaped
problem; the stopping test is unchanged, so every run ends at the same tolerances — compared on
ρ and the primal w = Φᵀ y α against the default start."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import svc_lowrank  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
dev = torch.device("cuda")
X, y, _ = make_hf_cohort(n, 17, seed=5, nan_frac=0.0)
Z = torch.as_tensor(X, device=dev)
Z = (Z - Z.mean(0)) / Z.std(0).clamp(min=1e-12)
g = torch.Generator().manual_seed(1)
idx = torch.randperm(Z.shape[0], generator=g)[:512].to(dev)
Phi, _ = svc_lowrank.nystrom_map(Z, idx, 1.0 / 17)
Phi = Phi.to(torch.float32).to(torch.float64)
yv = torch.as_tensor(np.where(y > 0.5, -1.0, 1.0), device=dev)
c = torch.where(yv > 0, 0.62, 2.5).to(torch.float64)
ref = None
for a0, nu0, nc in [(0.5, 1.0, 2), (0.1, 1.0, 2), (0.02, 1.0, 2), (0.005, 1.0, 2), (0.5, 10.0, 2), (0.5, 100.0, 2),
                    (0.1, 10.0, 2), (0.02, 0.1, 2), (0.5, 10.0, 3)]:
    svc_lowrank.IPM_A0, svc_lowrank.IPM_NU0, svc_lowrank.N_CORRECTORS = a0, nu0, nc
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a, rho, it = svc_lowrank.ipm_svc_dual(Phi, yv, c)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    w = Phi.T @ (yv * a)
    if ref is None:
        ref = (w, rho)
    dw = float((w - ref[0]).abs().max() / ref[0].abs().max())
    print(f"A0 {a0} NU0 {nu0} correctors {nc}: {it} iterations, {dt:.2f} s, rho {rho:.7f} (d {rho - ref[1]:+.1e}), "
          f"w rel diff {dw:.1e}", flush=True)

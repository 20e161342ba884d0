"""The interior point's convergence trajectory on a config-3-shaped problem (Table S1-shaped cohort,
17 selected features, Nyström map of 512 landmarks): per-iteration gap / residuals / step lengths
(HFENS_IPM_DEBUG=1 prints them)."""
import os
import sys

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
print("rank", Phi.shape, flush=True)
import time  # noqa: E402
for rep in range(int(os.environ.get("REPS", "1"))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a, rho, it = svc_lowrank.ipm_svc_dual(Phi, yv, c)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
w = Phi.t() @ (yv * a)
print(f"iterations {it} solve_s {dt:.3f} rho {rho:.9f} |w| {float(w.norm()):.9f} nsv {int((a > 0).sum())} "
      f"bound {int((a >= c * (1 - 1e-9)).sum())} correctors {svc_lowrank.N_CORRECTORS}", flush=True)

"""IPM iterations and time vs the number of Gondzio correctors on a config-3-shaped problem:
python scripts/ipm_correctors.py ROWS"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models import svc_lowrank  # noqa: E402
from hfens.models.smo import _expand  # noqa: E402
from hfens.models.svc import SVC  # noqa: E402

dev = torch.device("cuda")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
X, y = make_hf_cohort_device(n, 17, seed=2020, rows=(0, n), device=dev)
Z = ((X - X.mean(0)) / X.std(0, unbiased=False).clamp(min=1e-12)).to(torch.float64)
y_np = y.cpu().numpy().astype(np.float64)
gamma = 1.0 / (17 * float(Z.var(unbiased=False)))
cnt = np.bincount((y_np > 0.5).astype(np.int64), minlength=2).astype(np.float64)
probs, mt = _expand(0, y_np, gamma, n / (2 * cnt), SVC(class_weight="balanced", probability=True, random_state=2020))
pick = torch.randperm(n, generator=torch.Generator().manual_seed(7))[:512].numpy()
Phi, T = svc_lowrank.nystrom_map(Z, torch.as_tensor(np.sort(pick), device=dev), gamma)
yint = torch.as_tensor(np.where(y_np > 0.5, -1.0, 1.0), dtype=torch.float64, device=dev)
cvec = torch.where(yint > 0, torch.full_like(yint, mt["C0"]), torch.full_like(yint, mt["C1"]))
rows = torch.as_tensor(probs[0].rows, device=dev)
P, yy, cc = Phi[rows].contiguous(), yint[rows], cvec[rows]
ref = None
for k in (0, 1, 2, 3):
    svc_lowrank.N_CORRECTORS = k
    svc_lowrank.ipm_svc_dual(P[:20000], yy[:20000], cc[:20000])
    torch.cuda.synchronize()
    t = time.perf_counter()
    a, rho, it = svc_lowrank.ipm_svc_dual(P, yy, cc)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    w = (P * (yy * a)[:, None]).sum(0)
    if ref is None:
        ref = (w, rho)
    dw = float((w - ref[0]).abs().max() / ref[0].abs().max())
    print(f"correctors {k}: {it} iterations, {dt * 1e3:.0f} ms ({dt * 1e3 / it:.1f} ms/it), rho {rho:.6f}, "
          f"max rel diff of w vs 0 correctors {dw:.2e}", flush=True)

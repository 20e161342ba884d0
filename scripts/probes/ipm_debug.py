"""Interior-point SVC on a config-3-shaped problem (Table-S1 cohort, 17 scaled features, the
pipeline's landmark draw) with per-iteration state: python scripts/ipm_debug.py ROWS [native 0/1]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("HFENS_IPM_DEBUG", "1")
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models import svc_lowrank  # noqa: E402
from hfens.models.smo import _expand  # noqa: E402
from hfens.models.svc import SVC  # noqa: E402

dev = torch.device("cuda")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
X, y = make_hf_cohort_device(n, 17, seed=2020, rows=(0, n), device=dev)
Z = (X - X.mean(0)) / X.std(0, unbiased=False).clamp(min=1e-12)
Z = Z.to(torch.float64)
svc = SVC(class_weight="balanced", probability=True, random_state=2020)
y_np = y.cpu().numpy().astype(np.float64)
gamma = 1.0 / (17 * float(Z.var(unbiased=False)))
cnt = np.bincount((y_np > 0.5).astype(np.int64), minlength=2).astype(np.float64)
probs, mt = _expand(0, y_np, gamma, n / (2 * cnt), svc)
g = torch.Generator().manual_seed(2020 * 1000003 + n)
pick = torch.randperm(n, generator=g)[:512].numpy()
cls1 = y_np[pick] > 0.5
pick = np.concatenate([np.sort(pick[~cls1]), np.sort(pick[cls1])])
Phi, T = svc_lowrank.nystrom_map(Z, torch.as_tensor(pick, device=dev), gamma)
print("rank", T.shape[1], flush=True)
yint = torch.as_tensor(np.where(y_np > 0.5, -1.0, 1.0), dtype=torch.float64, device=dev)
cvec = torch.where(yint > 0, torch.full_like(yint, mt["C0"]), torch.full_like(yint, mt["C1"]))
p = probs[0]
rows = torch.as_tensor(p.rows, device=dev)
a, rho, it = svc_lowrank.ipm_svc_dual(Phi[rows], yint[rows], cvec[rows])
print("done", it, rho, flush=True)

"""LassoCV (cv=10, 100 alphas) on the headline cohort alone on the device: time of the fit and of
the lasso_cd_path launches (events), with and without the speculative refit, and the sweep counts."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import lasso as L  # noqa: E402

dev = torch.device("cuda")
X, y, _ = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.0)
X = torch.as_tensor(X, device=dev)
y = torch.as_tensor(y, device=dev)
orig = L.LassoCV._solve
rec = []


def timed(self, Gs, qs, yys, ns, grid):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = orig(self, Gs, qs, yys, ns, grid)
    e1.record()
    rec.append((int(Gs.shape[0]), e0, e1))
    return out


L.LassoCV._solve = timed
for spec in (True, False):
    L.SPECULATIVE_REFIT = spec
    for rep in range(6):
        rec.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = L.LassoCV(cv=10, random_state=2020).fit(X, y)
        torch.cuda.synchronize()
        wall = 1e3 * (time.perf_counter() - t0)
        if rep >= 3:
            print(f"spec={spec} wall {wall:.2f} ms; launches " +
                  ", ".join(f"P={p}: {a.elapsed_time(b):.3f} ms" for p, a, b in rec), flush=True)

"""Cooperative-SMO time vs members per problem for a rank's share of the bench's 36 problems:
with N ranks each solves ~36/N problems (LPT), so more CUs per problem are free.  Solves the
problems of the LAST k fits (k=1: the full fit's 5 Platt folds + final 10k problem) for several
member counts and prints ms per batch and µs per pair of the largest problem."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo  # noqa: E402
from hfens.models.model_selection import fold_masks, stratified_kfold_test_folds  # noqa: E402
from hfens.models.svc import SVC  # noqa: E402

dev = torch.device("cuda")
n = 10000
X, y, _ = make_hf_cohort(n, 17, seed=3, nan_frac=0.0)
X = torch.as_tensor(X, device=dev)
y = torch.as_tensor(y, device=dev)
masks = fold_masks(stratified_kfold_test_folds(y.cpu().numpy(), 5), 5, device=dev)
Zs, ys = [], []
for m in masks:
    r = torch.nonzero(m).squeeze(1)
    Xm = X[r]
    Zs.append((Xm - Xm.mean(0)) / Xm.std(0, unbiased=False))
    ys.append(y[r])
svc = SVC(class_weight="balanced", probability=True, random_state=2020)
for k_fits in (int(a) for a in (sys.argv[1:] or ["1", "2", "6"])):
    probs = []
    for f in range(6 - k_fits, 6):
        yn = ys[f].cpu().numpy()
        cnt = np.bincount((yn > 0.5).astype(np.int64), minlength=2).astype(np.float64)
        pr, _ = smo._expand(f, yn, 1.0 / (17 * float(Zs[f].var(unbiased=False))), yn.shape[0] / (2 * cnt), svc)
        probs += pr
    for W in (3, 4, 5, 6, 8, 12, 16):
        smo._COOP_MAX_W = W
        smo.COOP_RESERVE_CUS = 0
        ts = []
        for rep in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            sol = smo._solve_device(probs, Zs, dev, 1e-3)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        its = max(int(sol[id(p)][2]) for p in probs if p.rows is not None)
        dt = sorted(ts)[1]
        print(f"fits {k_fits} problems {len(probs)} W={smo.LAST_SMO_INFO.get('members')}: {dt * 1e3:7.1f} ms, "
              f"{dt * 1e6 / its:5.2f} us/pair (max iters {its})", flush=True)

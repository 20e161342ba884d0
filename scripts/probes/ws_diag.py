"""Diagnose the working-set SMO on the bench's SVC stage (10k rows, 36 problems)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from hfens.io.synth import make_hf_cohort
from hfens.models import smo
from hfens.models.svc import SVC
from hfens.models.stack_trainer import fit_base_batch  # noqa: F401  (import check)

import os
dev = torch.device("cuda")
N = int(os.environ.get("WS_DIAG_ROWS", "10000"))
X, y, _ = make_hf_cohort(N, 17, seed=2020, nan_frac=0.0)
X = torch.as_tensor(X, device=dev)
y = torch.as_tensor(y, device=dev)
Z = (X - X.mean(0)) / X.std(0, unbiased=False)
# 6 fits like the stack: 5 OOF folds (8k) + full (10k)
folds = torch.arange(N, device=dev) % 5
Zs = [Z[folds != k] for k in range(5)] + [Z]
ys = [y[folds != k] for k in range(5)] + [y]
nf = int(os.environ.get("WS_DIAG_FITS", "6"))   # the last nf fits (1 = the full-data fit: 6 problems)
Zs, ys = Zs[-nf:], ys[-nf:]
for spec in sys.argv[1:] or ["exact", "ws:0.1"]:
    solver, _, frac = spec.partition(":")
    smo.SOLVER = solver
    if frac:
        smo.WS_INNER_FRAC = float(frac)
    for rep in range(int(os.environ.get("WS_DIAG_REPS", "2"))):
        svcs = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in Zs]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        smo.fit_svc_batch(svcs, Zs, ys)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"{spec}: {1000 * dt:.1f} ms  n_iter={[s.n_iter_ for s in svcs]}  {smo.LAST_SMO_INFO}", flush=True)
    if solver == "exact" and smo.LAST_SMO_PROF:
        pr = smo.LAST_SMO_PROF
        k = int(np.argmax(pr["iters"]))
        it = max(1, int(pr["iters"][k]))
        names = pr.get("names", ["step2", "r2", "pair", "update", "r1"])
        print(f"  largest problem l={pr['l'][k]} iters={it}: cycles/iter " +
              ", ".join(f"{nm} {v / it:.0f}" for nm, v in zip(names, pr["phases"][k])))
    if solver == "ws":
        st = smo.LAST_WS_STATS
        print("  outer: max", int(st["outer"].max()), "mean", float(st["outer"].mean()))
        print("  inner: max", int(st["inner"].max()), "mean", float(st["inner"].mean()))
        k = int(np.argmax(st["outer"]))
        o = max(1, int(st["outer"][k]))
        print(f"  slowest problem: outer {o}, cycles/outer select {st['cyc_select'][k] / o:.0f} "
              f"build {st['cyc_build'][k] / o:.0f} inner {st['cyc_inner'][k] / o:.0f} "
              f"(inner/outer {st['inner'][k] / o:.1f}); select = p0 {st['cyc_p0'][k] / o:.0f} "
              f"p1 {st['cyc_p1'][k] / o:.0f} p2 {st['cyc_p2'][k] / o:.0f} + compaction")

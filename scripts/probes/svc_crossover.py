"""Exact working-set SMO (no Gram, svm_ws.hip K-cached rounds) vs the Nyström + interior-point
approximation (svc_lowrank) for one probability SVC fit (5 Platt folds + the final problem) at
growing row counts: wall time, rounds / pairs, held-out AUROC and decision-value agreement
(VERDICT r3 next #3).  Usage: python scripts/probes/svc_crossover.py 40000 100000 ...
Prints one JSON line per (rows, solver)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo  # noqa: E402
from hfens.models.svc import SVC  # noqa: E402
from hfens.utils import metrics  # noqa: E402

dev = torch.device("cuda")
for rows in [int(a) for a in sys.argv[1:]] or [40000]:
    X, y, _ = make_hf_cohort(rows, 17, seed=rows, nan_frac=0.0)
    Xt, yt, _ = make_hf_cohort(20000, 17, seed=rows + 1, nan_frac=0.0)
    mu, sd = X.mean(0), X.std(0)
    sd = np.where(sd > 0, sd, 1.0)
    Z = torch.as_tensor((X - mu) / sd, device=dev)
    Zt = torch.as_tensor((Xt - mu) / sd, device=dev)
    yd = torch.as_tensor(y, device=dev)
    dec = {}
    from hfens.models import svc_lowrank
    solvers = os.environ.get("SOLVERS", "ws,lowrank").split(",")
    for solver in solvers:
        # ws = exact working set (cascade-seeded), ws_cold = exact without the seed,
        # lowrankN = Nyström + IPM with N landmarks (lowrank = the default count)
        smo.SOLVER = "ws" if solver.startswith("ws") else "lowrank"
        smo.CASCADE = solver != "ws_cold"
        if solver.startswith("lowrank") and solver != "lowrank":
            svc_lowrank.N_LANDMARKS = int(solver[7:])
        for rep in range(2):   # second fit timed (first: allocations, code objects)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = SVC(class_weight="balanced", probability=True, random_state=2020).fit(Z, yd)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        d = m.decision_function(Zt).double().cpu().numpy()
        p = m.predict_proba(Zt)[:, 1].double().cpu().numpy()
        dec[solver] = d
        out = dict(rows=rows, solver=solver, fit_s=round(dt, 3),
                   auroc=round(float(metrics.evaluate(torch.as_tensor(yt), torch.as_tensor(p))["auroc"]), 5))
        if solver.startswith("ws"):
            st = smo.LAST_WS_STATS
            out.update(rounds_max=int(st["outer"].max()), pairs_max=int(st["inner"].max()),
                       gap_max=float(st["gap"].max()))
        print(json.dumps(out), flush=True)
    ref = solvers[0]
    for other in solvers[1:]:
        c = np.corrcoef(dec[ref], dec[other])[0, 1]
        print(json.dumps(dict(rows=rows, ref=ref, other=other, decision_corr=round(float(c), 6),
                              max_abs_diff=round(float(np.abs(dec[ref] - dec[other]).max()), 5))), flush=True)

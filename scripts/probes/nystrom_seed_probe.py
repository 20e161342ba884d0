"""Nyström-seeded exact SVC at 300k–1M points.

One ``SVC(probability=True, class_weight="balanced")`` fit (5 Platt folds + the final problem) by
the exact working-set solver (svm_ws.hip, K-cached rounds past 16k points) started three ways:
  cold     α = 0;
  cascade  the cascade seed the solver uses today (class-stratified parts solved loosely);
  nystrom  every problem's reduced-set dual solved by the interior point (svc_lowrank: 512
           landmarks, the Nyström map, ipm_svc_dual), its α projected onto the EXACT problem's box
           and equality constraints (:func:`project`), and handed to the solver as its seed.
Records wall time (seed time separately), rounds / pairs of the largest problem, its final gap,
held-out AUROC and decision-value agreement with the first variant.  One JSON line per
(rows, variant).  Usage: python scripts/probes/nystrom_seed_probe.py 300000 [1000000]
VARIANTS=cold,cascade,nystrom (default)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo, svc_lowrank  # noqa: E402
from hfens.models.svc import SVC  # noqa: E402
from hfens.utils import metrics  # noqa: E402

dev = torch.device("cuda")
_orig_seed = smo._cascade_seed
SEED_INFO = {}


def project(a, y, c, rel=1e-5, iters=100):
    """α onto the exact problem's box and equality constraints, every value either AT a bound or
    clearly inside (≥ rel·C from it).  The interior point returns every α strictly inside (0, C),
    most within 1e-8 of a bound: the solver's f64 selection keys see such a point as free while its
    f32 inner solve sees it at the bound, so a working set of them holds no f32-violating pair and
    the round reports "done" at a large gap (r6ag / r6ah, first run).  So: snap to the bounds within
    rel·C, then restore Σ y α = 0 by a shift τ of the free values only (clipped to [rel·C, (1−rel)·C],
    bisection on τ)."""
    a = torch.minimum(a.clamp(min=0.0), c)
    lo_t, hi_t = rel * c, (1.0 - rel) * c
    at0, atc = a <= lo_t, a >= hi_t
    a = torch.where(at0, torch.zeros_like(a), torch.where(atc, c, a))
    free = ~(at0 | atc)
    base = float((y * a)[~free].sum())
    af, yf, lf, hf = a[free], y[free], lo_t[free], hi_t[free]
    lo, hi = -float(c.max()), float(c.max())
    for _ in range(iters):
        t = 0.5 * (lo + hi)
        h = base + float((yf * torch.minimum(torch.maximum(af - t * yf, lf), hf)).sum())
        if h > 0:
            lo = t
        else:
            hi = t
    t = 0.5 * (lo + hi)
    a = a.clone()
    a[free] = torch.minimum(torch.maximum(af - t * yf, lf), hf)
    return a


def nystrom_seed(E, live, zcat, aoffs, F, device, s, max_iter_cap=None):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    seed = torch.zeros(aoffs[-1], dtype=torch.float64, device=device)
    its, resid = [], []
    for k, p in enumerate(live):
        a0, l = aoffs[k], p.l
        Zk = zcat[a0:a0 + l].to(torch.float64)
        y = torch.ones(l, dtype=torch.float64, device=device)
        y[p.npos:] = -1.0
        c = torch.where(y > 0, torch.full_like(y, p.Cp), torch.full_like(y, p.Cn))
        g = torch.Generator().manual_seed(2020 * 1000003 + l)
        idx = torch.randperm(l, generator=g)[:min(svc_lowrank.N_LANDMARKS, l)].sort().values.to(device)
        Phi, _ = svc_lowrank.nystrom_map(Zk, idx, float(p.gamma))
        a, _, it = svc_lowrank.ipm_svc_dual(Phi.contiguous(), y, c)
        ap = project(a, y, c)
        resid.append(float((y * ap).sum()))
        its.append(int(it))
        seed[a0:a0 + l] = ap
    torch.cuda.synchronize()
    SEED_INFO.update(seed_s=round(time.perf_counter() - t0, 3), ipm_iters=its,
                     max_abs_y_alpha=max(abs(r) for r in resid),
                     seed_free_frac=round(float(((seed > 0) & (seed < seed.max())).double().mean()), 4))
    return seed


variants = os.environ.get("VARIANTS", "cold,cascade,nystrom").split(",")
for rows in [int(a) for a in sys.argv[1:]] or [300000]:
    X, y, _ = make_hf_cohort(rows, 17, seed=rows, nan_frac=0.0)
    Xt, yt, _ = make_hf_cohort(20000, 17, seed=rows + 1, nan_frac=0.0)
    mu, sd = X.mean(0), X.std(0)
    sd = np.where(sd > 0, sd, 1.0)
    Z = torch.as_tensor((X - mu) / sd, device=dev)
    Zt = torch.as_tensor((Xt - mu) / sd, device=dev)
    yd = torch.as_tensor(y, device=dev)
    dec = {}
    smo.SOLVER = "ws"
    for v in variants:
        smo.CASCADE = v != "cold"
        smo._cascade_seed = nystrom_seed if v == "nystrom" else _orig_seed
        SEED_INFO.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = SVC(class_weight="balanced", probability=True, random_state=2020).fit(Z, yd)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        d = m.decision_function(Zt).double().cpu().numpy()
        p = m.predict_proba(Zt)[:, 1].double().cpu().numpy()
        dec[v] = d
        st = smo.LAST_WS_STATS
        k = int(st["inner"].argmax())
        out = dict(rows=rows, variant=v, fit_s=round(dt, 3), rounds_max=int(st["outer"].max()),
                   pairs_max=int(st["inner"].max()), gap_of_max=float(st["gap"][k]),
                   gap_max=float(st["gap"].max()),
                   auroc=round(float(metrics.evaluate(torch.as_tensor(yt), torch.as_tensor(p))["auroc"]), 5),
                   **SEED_INFO)
        print(json.dumps(out), flush=True)
    ref = variants[0]
    for other in variants[1:]:
        print(json.dumps(dict(rows=rows, ref=ref, other=other,
                              decision_corr=round(float(np.corrcoef(dec[ref], dec[other])[0, 1]), 6),
                              max_abs_diff=round(float(np.abs(dec[ref] - dec[other]).max()), 5))), flush=True)
    smo._cascade_seed = _orig_seed

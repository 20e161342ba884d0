"""Tiny end-to-end check of the flagship path on one device (used by
``__graft_entry__.smoke``): checkpoint inference through the HIP kernels and one
small ensemble training step (the bench's development fit at 400 rows)."""
from __future__ import annotations

import torch


def run_smoke(dev) -> None:
    from ..cli.predict_hf import PATIENT_PARAMS
    from ..io.checkpoint import load_checkpoint
    clf = load_checkpoint(device=dev)
    x = torch.tensor([[float(v) for v in PATIENT_PARAMS.values()]], dtype=torch.float64, device=dev)
    p = float(clf.predict_proba(x)[0, 1])
    assert abs(p - 0.2709003) < 1e-5, p
    auc = train_smoke(dev)
    torch.cuda.synchronize(dev)
    print(f"[smoke] ok  P(default patient)={p:.6f}  tiny develop() held-out AUROC={auc:.3f}")


def train_smoke(dev, rows: int = 400, features: int = 24) -> float:
    """One tiny development fit on ``dev`` through the HIP kernels: KNN impute → LassoCV top-17 →
    stacking fit (36 SMO problems, 6 GBDTs, 6 L1-LRs, meta-LR) → held-out AUROC."""
    from ..io.synth import make_hf_cohort
    from ..pipeline import develop
    Xd, yd, names = make_hf_cohort(rows, features, seed=7, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(rows, features, seed=8, nan_frac=0.02)
    res = develop(Xd, yd, Xs, ys, names, device=dev, evaluate=True)
    auc = float(res.scores["auroc"])
    assert 0.5 < auc <= 1.0 and len(res.selected_names) == 17, (auc, res.selected_names)
    return auc

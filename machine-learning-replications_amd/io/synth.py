"""Synthetic HCM cohorts shaped like the reference's private data.

The reference trains on private MATLAB tables (``train_ensemble_public.py:36,39``)
that are not shipped.  Supplementary Table S1 (reference ``Table 1.DOCX``) gives
the cohort statistics of all 64 candidate variables over 1,427 patients; this
module samples independent columns with those marginals (binary prevalence,
Gaussian mean±SD clipped at 0, or ordinal ranges), keeps the cohort's
NYHA = 1 + Dyspnea collinearity, draws ~2 % missing
values, and labels rows with a sparse logistic model whose coefficients on the
17 model features are the shipped L1-LR's (checkpoint ``estimators_[2].coef_``)
and ~20 % prevalence (141/713 in the checkpoint).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np
import torch

# (name, kind, params) — kind: "bin" p | "gauss" (mean, sd) | "ord" (lo, hi, p_nonzero)
TABLE_S1: List[Tuple[str, str, tuple]] = [
    ("Gender", "bin", (0.69,)),
    ("Age at HCM diagnosis", "gauss", (45.0, 18.0)),
    ("Obstructive HCM", "bin", (0.52,)),
    ("Massive hypertrophy", "bin", (0.06,)),
    ("NSVT on holter", "bin", (0.10,)),
    ("Syncope", "bin", (0.10,)),
    ("Dyspnea", "bin", (0.45,)),
    ("Chest pain", "bin", (0.18,)),
    ("Fatigue", "bin", (0.14,)),
    ("Presyncope", "bin", (0.05,)),
    ("Palpitations", "bin", (0.14,)),
    ("NYHA functional class", "nyha", ()),
    ("ICD", "bin", (0.11,)),
    ("Appropriate ICD shocks", "bin", (0.01,)),
    ("Number of ICD shocks", "ord", (0, 8, 0.02)),
    ("Permanent pace maker", "bin", (0.015,)),
    ("Mitral valve surgery", "bin", (0.002,)),
    ("VT ablation", "bin", (0.003,)),
    ("CABG", "bin", (0.004,)),
    ("Stents", "bin", (0.03,)),
    ("Cardioversion", "bin", (0.045,)),
    ("Number of DC cardioversions", "ord", (0, 4, 0.045)),
    ("AF ablation", "bin", (0.011,)),
    ("Number of AF ablations", "ord", (0, 3, 0.011)),
    ("Recurrent AF after ablation", "bin", (0.009,)),
    ("Atrial fibrillation", "bin", (0.14,)),
    ("Resuscitated cardiac arrest", "bin", (0.017,)),
    ("Hypertension", "bin", (0.32,)),
    ("Coronary artery disease", "bin", (0.055,)),
    ("Prior myocardial infarction", "bin", (0.015,)),
    ("Stroke", "bin", (0.022,)),
    ("Type of stroke", "ord", (0, 2, 0.022)),
    ("Family history of SCD", "bin", (0.11,)),
    ("FH SCD relation", "ord", (0, 4, 0.11)),
    ("FH SCD multiple relatives", "bin", (0.04,)),
    ("Family history of HCM", "bin", (0.26,)),
    ("FH end stage HCM", "bin", (0.03,)),
    ("FH heart transplant", "bin", (0.018,)),
    ("Beta blocker", "bin", (0.57,)),
    ("Calcium channel blockers", "bin", (0.20,)),
    ("Disopyramide", "bin", (0.014,)),
    ("ACE inhibitor or ARB", "bin", (0.22,)),
    ("Spironolactone", "bin", (0.011,)),
    ("Diuretic", "bin", (0.11,)),
    ("Amiodarone", "bin", (0.019,)),
    ("Coumadin", "bin", (0.056,)),
    ("Aspirin", "bin", (0.28,)),
    ("Statin", "bin", (0.32,)),
    ("Novel anti-coagulation", "bin", (0.036,)),
    ("Other anti-arrhythmic", "bin", (0.031,)),
    ("Other cardiac medications", "bin", (0.027,)),
    ("Maximum LV wall thick (mm)", "gauss", (19.0, 5.0)),
    ("Septal anterior motion", "bin", (0.68,)),
    ("LVOT gradient (mmHg)", "gauss", (19.0, 35.0)),
    ("Mid-cavity gradient", "gauss", (3.0, 12.0)),
    ("Mitral regurgitation", "ord", (0, 4, 0.45)),
    ("LV ejection fraction (%)", "gauss", (64.0, 5.0)),
    ("LA diameter (mm)", "gauss", (40.0, 7.0)),
    ("LVEDD (mm)", "gauss", (42.0, 7.0)),
    ("LVESD (mm)", "gauss", (27.0, 6.0)),
    ("Severe aortic stenosis", "bin", (0.006,)),
    ("Apical HCM", "bin", (0.11,)),
    ("Apical aneurysm", "bin", (0.03,)),
    ("End-stage HCM", "bin", (0.018,)),
]

# The 17 model features (reference predict_hf.py:5-27 order) → Table S1 rows.
MODEL_FEATURES = ["Obstructive HCM", "Gender", "Syncope", "Dyspnea", "Fatigue", "Presyncope",
                  "NYHA functional class", "Atrial fibrillation", "Hypertension", "Beta blocker",
                  "Calcium channel blockers", "ACE inhibitor or ARB", "Coumadin",
                  "Maximum LV wall thick (mm)", "Septal anterior motion", "Mitral regurgitation",
                  "LV ejection fraction (%)"]
# shipped L1-LR coefficients (raw units) for the label model
MODEL_COEF = [1.125, -0.249, 0.390, 1.195, 0.562, 1.424, 0.421, 0.204, -0.218, 0.587, 0.361,
              -0.416, 1.227, 0.042, 0.772, 0.196, -0.065]


def feature_order(n_features: int) -> List[str]:
    """First the 17 model features, then the remaining Table S1 rows in table order."""
    names = list(MODEL_FEATURES)
    names += [r[0] for r in TABLE_S1 if r[0] not in MODEL_FEATURES]
    if not 1 <= n_features <= len(names):
        raise ValueError(f"n_features must be in [1, {len(names)}]")
    return names[:n_features]


def _column(rng, kind, params, n, dysp=None):
    if kind == "bin":
        return (rng.random(n) < params[0]).astype(np.float64)
    if kind == "gauss":
        m, s = params
        v = np.round(rng.normal(m, s, n), 1)
        return np.clip(v, 0.0, None)
    if kind == "ord":
        lo, hi, p = params
        nz = rng.random(n) < p
        return np.where(nz, rng.integers(max(lo, 1), hi + 1, n), lo).astype(np.float64)
    if kind == "nyha":
        return 1.0 + dysp
    raise ValueError(kind)


def make_hf_cohort(n_rows: int, n_features: int = 40, seed: int = 0, nan_frac: float = 0.02,
                   prevalence: float = 0.2, signal: float = 2.5):
    """Return ``(X float64 [n, F] with NaNs, y float64 {0,1}, names)``."""
    rng = np.random.default_rng(seed)
    spec = {r[0]: r for r in TABLE_S1}
    names = feature_order(n_features)
    cols = {}
    cols["Dyspnea"] = _column(rng, "bin", spec["Dyspnea"][2], n_rows)
    full_names = feature_order(len(TABLE_S1))
    for nm in full_names:
        if nm in cols:
            continue
        kind, params = spec[nm][1], spec[nm][2]
        cols[nm] = _column(rng, kind, params, n_rows, dysp=cols["Dyspnea"])
    X = np.stack([cols[nm] for nm in names], axis=1)
    # label model: the shipped L1-LR on the 17 model features + weak effects of 5 others
    lin = np.zeros(n_rows)
    for nm, c in zip(MODEL_FEATURES, MODEL_COEF):
        v = cols[nm]
        lin += c * (v - v.mean())
    extra = [nm for nm in full_names if nm not in MODEL_FEATURES][:5]
    # fixed label model: every draw (dev / held-out / any seed) shares the same outcome model
    wts = np.random.default_rng(7919).normal(0, 0.3, len(extra))
    for nm, c in zip(extra, wts):
        v = cols[nm]
        lin += c * (v - v.mean()) / (v.std() + 1e-12)
    lin *= signal  # 2.5 → held-out AUROC ≈ 0.9 for a linear model
    # intercept for the requested prevalence (bisection on the mean probability)
    lo, hi = -20.0, 20.0
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        if (1 / (1 + np.exp(-(lin + mid)))).mean() > prevalence:
            hi = mid
        else:
            lo = mid
    p = 1 / (1 + np.exp(-(lin + 0.5 * (lo + hi))))
    y = (rng.random(n_rows) < p).astype(np.float64)
    if nan_frac > 0:
        miss = rng.random(X.shape) < nan_frac
        X = X.copy()
        X[miss] = np.nan
    return X, y, names


def make_dev_select(n_rows: int, n_features: int = 40, seed: int = 2020, nan_frac: float = 0.02):
    """Development + independent held-out ("model select") draws of equal size
    (reference ``train_ensemble_public.py:36,39``)."""
    Xd, yd, names = make_hf_cohort(n_rows, n_features, seed, nan_frac)
    Xs, ys, _ = make_hf_cohort(n_rows, n_features, seed + 1, nan_frac)
    return Xd, yd, Xs, ys, names


# ----------------------------------------------------------------------------- device generator
_CHUNK = 1 << 16


def _label_model(n_features: int, seed: int):
    """Coefficients (per model column, on standardized columns) and the intercept for ~20 %
    positives — the same structure as ``make_hf_cohort``'s label model."""
    names = feature_order(n_features)
    spec = {r[0]: r for r in TABLE_S1}
    coef = np.zeros(n_features)
    for i, nm in enumerate(names):
        if nm in MODEL_FEATURES:
            coef[i] = MODEL_COEF[MODEL_FEATURES.index(nm)]
    extra = [i for i, nm in enumerate(names) if nm not in MODEL_FEATURES][:5]
    coef[extra] = np.random.default_rng(7919).normal(0, 0.3, len(extra))
    mean = np.zeros(n_features)
    sd = np.ones(n_features)
    for i, nm in enumerate(names):
        kind, params = spec[nm][1], spec[nm][2]
        if kind == "bin":
            mean[i], sd[i] = params[0], np.sqrt(params[0] * (1 - params[0]))
        elif kind == "gauss":
            mean[i], sd[i] = params
        elif kind == "ord":
            lo, hi, p = params
            mean[i] = (1 - p) * lo + p * (max(lo, 1) + hi) / 2
            sd[i] = max(1e-3, np.sqrt(p) * (hi - lo) / 2)
        else:   # nyha = 1 + dyspnea
            pd_ = spec["Dyspnea"][2][0]
            mean[i], sd[i] = 1 + pd_, np.sqrt(pd_ * (1 - pd_))
    # model features enter unstandardized in make_hf_cohort (× signal 2.5); extras standardized
    scale = np.where([nm in MODEL_FEATURES for nm in names], 1.0, 1.0 / sd)
    w = 2.5 * coef * scale
    return names, w, mean


def make_hf_cohort_device(n_total: int, n_features: int = 40, seed: int = 0, rows=None, device="cuda",
                          prevalence: float = 0.2):
    """Table-S1-shaped rows generated ON the device, without NaNs: ``(X f32 [e-s, F], y f32)``
    for global rows ``rows = (s, e)`` of an ``n_total``-row cohort.  Rows come in fixed 64k-row
    chunks each seeded by (seed, chunk), so any row range — a rank's data-parallel shard — is
    the same slice of the same global cohort whatever the number of ranks (strong scaling)."""
    s, e = (0, n_total) if rows is None else rows
    names, w, mean = _label_model(n_features, seed)
    spec = {r[0]: r for r in TABLE_S1}
    kinds = [(spec[nm][1], spec[nm][2]) for nm in names]
    dys = names.index("Dyspnea") if "Dyspnea" in names else None
    wt = torch.as_tensor(w, dtype=torch.float32, device=device)
    mu = torch.as_tensor(mean, dtype=torch.float32, device=device)
    # intercept for the prevalence: bisection on a fixed 64k probe chunk
    probe_X, _ = _device_chunk(kinds, dys, n_features, seed, -1, _CHUNK, device, None, 0.0)
    lin = (probe_X - mu) @ wt
    lo, hi = -20.0, 20.0
    for _ in range(50):
        mid = 0.5 * (lo + hi)
        if float(torch.sigmoid(lin + mid).mean()) > prevalence:
            hi = mid
        else:
            lo = mid
    b0 = 0.5 * (lo + hi)
    Xs, ys = [], []
    for c in range(s // _CHUNK, (e + _CHUNK - 1) // _CHUNK):
        Xc, yc = _device_chunk(kinds, dys, n_features, seed, c, _CHUNK, device, (wt, mu), b0)
        c0 = c * _CHUNK
        a, z = max(s, c0) - c0, min(e, c0 + _CHUNK) - c0
        Xs.append(Xc[a:z])
        ys.append(yc[a:z])
    return torch.cat(Xs), torch.cat(ys)


def _device_chunk(kinds, dys, F, seed, c, m, device, lab, b0):
    g = torch.Generator(device=device).manual_seed((seed * 1_000_003 + c + 17) & 0x7FFFFFFFFFFFFFFF)
    X = torch.empty(m, F, dtype=torch.float32, device=device)
    U = torch.rand(m, F, generator=g, device=device)
    N = torch.randn(m, F, generator=g, device=device)
    for j, (kind, params) in enumerate(kinds):
        if kind == "bin":
            X[:, j] = (U[:, j] < params[0]).float()
        elif kind == "gauss":
            X[:, j] = torch.clamp(torch.round((params[0] + params[1] * N[:, j]) * 10) / 10, min=0.0)
        elif kind == "ord":
            lo_, hi_, p = params
            k = torch.floor(N[:, j].abs() * 1e4 % (hi_ - max(lo_, 1) + 1)) + max(lo_, 1)
            X[:, j] = torch.where(U[:, j] < p, k, torch.full_like(k, float(lo_)))
    for j, (kind, _) in enumerate(kinds):
        if kind == "nyha":
            X[:, j] = 1.0 + (X[:, dys] if dys is not None else 0.0)
    y = None
    if lab is not None:
        wt, mu = lab
        p = torch.sigmoid((X - mu) @ wt + b0)
        y = (torch.rand(m, generator=g, device=device) < p).float()
    return X, y

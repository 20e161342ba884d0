"""Single-patient (or batched) HF-progression probability from ``hf_predict_model.pkl``.

Same no-argument contract as the reference ``predict_hf.py:1-40``: the 17 clinical
inputs (ordered as the model's columns, ``predict_hf.py:5-27``) default to the
shipped example patient and the probability is printed between ``#`` rules.
Additions: ``--set NAME=VALUE`` overrides, ``--csv`` batched scoring, ``--device``
(``cuda`` runs the gfx950 kernels), ``--model`` path.
"""
from __future__ import annotations

import argparse
import sys
from collections import OrderedDict

import numpy as np
import torch

# Column order of the shipped model (reference predict_hf.py:5-27).
PATIENT_PARAMS = OrderedDict([
    ("Obstructive HCM", 1),          # 0 or 1
    ("Gender", 1),                   # Male:0 or Female: 1
    ("Syncope", 0),                  # 0 or 1
    ("Dyspnea", 0),                  # 0 or 1
    ("Fatigue", 1),                  # 0 or 1
    ("Presyncope", 0),               # 0 or 1
    ("NYHA_Class", 1),               # 1 or 2
    ("Atrial_Fibrillation", 1),      # 0 or 1
    ("Hypertension", 0),             # 0 or 1
    ("Beta_blocker", 0),             # 0 or 1
    ("Ca_Channel_Blockers", 0),      # 0 or 1
    ("ACEI_ARB", 0),                 # 0 or 1
    ("Coumadin", 0),                 # 0 or 1
    ("Max_Wall_Thick", 13),          # mm, echocardiography
    ("Septal_Anterior_Motion", 0),   # 0 or 1
    ("Mitral_Regurgitation", 0),     # 0..4
    ("Ejection_Fraction", 55),       # %, echocardiography
])


def format_probability(p1: float) -> str:
    bar = "###########################################"
    return f"{bar}\nProbability of progressive HF is: {100 * p1:.2f} %\n{bar}"


def predict_patient(params=None, model_path=None, device="cpu") -> float:
    from ..io.checkpoint import load_checkpoint
    params = PATIENT_PARAMS if params is None else params
    x = torch.tensor([[float(v) for v in params.values()]], dtype=torch.float64)
    clf = load_checkpoint(model_path, device=device)
    p = clf.predict_proba(x.to(device))
    return float(p[0, 1])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model", default=None, help="checkpoint path (default: assets/hf_predict_model.pkl)")
    ap.add_argument("--set", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("--csv", default=None, help="score every row of a CSV with the 17 columns")
    ap.add_argument("--device", default="cpu")
    a = ap.parse_args(argv)
    if a.csv:
        from ..io.checkpoint import load_checkpoint
        X = np.loadtxt(a.csv, delimiter=",", ndmin=2)
        clf = load_checkpoint(a.model, device=a.device)
        p = clf.predict_proba(torch.as_tensor(X, dtype=torch.float64, device=a.device))[:, 1]
        for v in p.cpu().tolist():
            print(f"{v:.6f}")
        return 0
    params = OrderedDict(PATIENT_PARAMS)
    for kv in a.set:
        k, v = kv.split("=", 1)
        if k not in params:
            print(f"unknown clinical variable {k!r}; expected one of {list(params)}", file=sys.stderr)
            return 2
        params[k] = float(v)
    print(format_probability(predict_patient(params, a.model, a.device)))
    return 0


if __name__ == "__main__":
    sys.exit(main())

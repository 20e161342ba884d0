"""Tiny end-to-end check of the flagship path on one device (used by
``__graft_entry__.smoke``): checkpoint inference through the HIP kernels and —
once available — one small ensemble training step."""
from __future__ import annotations

import torch


def run_smoke(dev) -> None:
    from ..cli.predict_hf import PATIENT_PARAMS
    from ..io.checkpoint import load_checkpoint
    clf = load_checkpoint(device=dev)
    x = torch.tensor([[float(v) for v in PATIENT_PARAMS.values()]], dtype=torch.float64, device=dev)
    p = float(clf.predict_proba(x)[0, 1])
    assert abs(p - 0.2709003) < 1e-5, p
    try:
        from .train_smoke import train_smoke
    except ImportError:
        train_smoke = None
    if train_smoke is not None:
        train_smoke(dev)
    torch.cuda.synchronize(dev)
    print(f"[smoke] ok  P(default patient)={p:.6f}")

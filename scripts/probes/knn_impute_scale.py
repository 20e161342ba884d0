"""Imputation at scale: KNNImputer(n_neighbors=1) fit + transform of an n-row Table S1-shaped cohort
on the device, timed per HFENS_KNN_MFMA mode (the matrix-core vs packed-FMA donor filter)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import imputer as imp_mod  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1"]
X, _, _ = make_hf_cohort(n, 40, seed=3, nan_frac=0.02)
Xt = torch.as_tensor(X, device="cuda")
out = {}
for mode in modes + modes:
    imp_mod.MFMA_FILTER = mode
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out[mode] = imp_mod.KNNImputer(n_neighbors=1).fit(Xt).transform(Xt)
    torch.cuda.synchronize()
    print(f"n={n} mode={mode}: {time.perf_counter() - t0:.3f} s", flush=True)
if len(modes) > 1:
    print("equal", torch.equal(out[modes[0]], out[modes[1]]), flush=True)

"""KNN imputation time on the GPU at large row counts (config 3's first stage):
python scripts/knn_probe.py ROWS [ROWS ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models.imputer import KNNImputer  # noqa: E402

dev = torch.device("cuda")
for n in (int(a) for a in sys.argv[1:] or ["100000"]):
    X, _, _ = make_hf_cohort(n, 40, seed=5, nan_frac=0.02)
    Xd = torch.as_tensor(X, device=dev)
    imp = KNNImputer(n_neighbors=1).fit(Xd)
    out = imp.transform(Xd)
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = imp.transform(Xd)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    rows_missing = int(torch.isnan(Xd).any(1).sum())
    print(f"rows {n}: transform {dt * 1e3:.1f} ms, receivers {rows_missing}, "
          f"{rows_missing * n / dt / 1e9:.2f} G receiver-donor pairs/s, nan left {int(torch.isnan(out).sum())}",
          flush=True)

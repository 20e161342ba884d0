"""How many receivers the KNN f64 refine re-scans (HFENS_KNN_DEBUG=1): the bench cohort's dev rows."""
import os
import sys
import time

os.environ["HFENS_KNN_DEBUG"] = "1"
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import imputer  # noqa: E402

dev = torch.device("cuda")
X, _, _ = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xt = torch.as_tensor(X, device=dev)
for rep in range(3):
    imputer.LAST_REFINE.clear()
    imp = imputer.KNNImputer(n_neighbors=1).fit(Xt)
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = imp.transform(Xt)
    torch.cuda.synchronize()
    print(f"rep {rep}: transform {1e3 * (time.perf_counter() - t):.2f} ms; (receivers, pass-0 re-scanned, pass-1, ‖m‖) = {imputer.LAST_REFINE}", flush=True)

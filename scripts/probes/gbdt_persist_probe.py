"""Per-stage cost of the GBDT stage loop, launch per stage vs the persistent loop (one launch, a
device grid barrier between stages): fit wall time and stage-loop device time at 125k rows (one
8-GPU share of 1M) and 1M rows, 1 and 5 models, 100 stumps."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models import hist_gbdt  # noqa: E402
from hfens.models.gbdt import GradientBoostingClassifier  # noqa: E402
from hfens.models.hist_gbdt import fit_gbdt_batch  # noqa: E402

dev = torch.device("cuda", 0)
T = int(os.environ.get("PROBE_TREES", "100"))
out = {}
for rows in (125_000, 1_000_000):
    X, y = make_hf_cohort_device(rows, 40, seed=7, rows=(0, rows), device=dev)
    for B in (1, 5):
        for mode in ("0", "1"):
            hist_gbdt.PERSIST = mode
            wall, loop = [], []
            for rep in range(5):
                ms = [GradientBoostingClassifier(n_estimators=T, max_depth=1, random_state=1 + k) for k in range(B)]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fit_gbdt_batch(ms, X, y)
                torch.cuda.synchronize()
                if rep >= 2:
                    wall.append(time.perf_counter() - t0)
                    e0, e1 = hist_gbdt.GRAPH_INFO["loop_events"]
                    loop.append(e0.elapsed_time(e1))
            key = f"{rows}_B{B}_persist{mode}"
            out[key] = dict(fit_ms=round(1e3 * sorted(wall)[1], 3), loop_ms=round(sorted(loop)[1], 3),
                            loop_us_per_stage=round(1e3 * sorted(loop)[1] / (T + 2), 2),
                            persist=hist_gbdt.GRAPH_INFO.get("persist"))
            print(key, out[key], flush=True)
    del X, y
print(json.dumps({"trees": T, "results": out}))

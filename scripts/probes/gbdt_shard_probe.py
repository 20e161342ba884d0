"""Where a GBDT fit's time goes at an 8-GPU shard (125k rows) vs the whole 1M rows (VERDICT r2
#1, Weak #7): fit wall time, stage-loop device time (events around the loop), per stage; with
no group and with a one-rank group whose per-stage sum goes through the IPC peer kernel
(parallel/xgmi.py) — the per-stage cost of the peer reduction at world 1."""
import json
import os
import sys
import tempfile
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models import hist_gbdt  # noqa: E402
from hfens.models.gbdt import GradientBoostingClassifier  # noqa: E402
from hfens.models.hist_gbdt import fit_gbdt_batch  # noqa: E402
from hfens.utils import timing  # noqa: E402

dev = torch.device("cuda", 0)
T = int(os.environ.get("PROBE_TREES", "100"))
store = tempfile.mktemp(prefix="hfens_pg_")
dist.init_process_group("gloo", init_method=f"file://{store}", rank=0, world_size=1)
g = dist.group.WORLD
out = {}
for rows in (125_000, 1_000_000):
    X, y = make_hf_cohort_device(rows, 40, seed=7, rows=(0, rows), device=dev)
    for B in (1, 5):
        for name, group in (("nogroup", None), ("xgmi_world1", g)):
            wall, loop = [], []
            for rep in range(5):
                ms = [GradientBoostingClassifier(n_estimators=T, max_depth=1, random_state=1 + k) for k in range(B)]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fit_gbdt_batch(ms, X, y, group=group)
                torch.cuda.synchronize()
                if rep >= 2:
                    wall.append(time.perf_counter() - t0)
                    e0, e1 = hist_gbdt.GRAPH_INFO["loop_events"]
                    loop.append(e0.elapsed_time(e1))
            key = f"{rows}_B{B}_{name}"
            out[key] = dict(fit_ms=round(1e3 * sorted(wall)[1], 3), loop_ms=round(sorted(loop)[1], 3),
                            loop_us_per_stage=round(1e3 * sorted(loop)[1] / (T + 2), 2),
                            xgmi_per_stage=hist_gbdt.COLLECTIVES.get("xgmi_per_stage"),
                            rccl_per_stage=hist_gbdt.COLLECTIVES.get("per_stage"),
                            graph_units=hist_gbdt.GRAPH_INFO.get("units"))
            print(key, out[key], flush=True)
    del X, y
from hfens.parallel import xgmi  # noqa: E402
xgmi.release_all()
dist.destroy_process_group()
print(json.dumps({"trees": T, "results": out}))

"""Per-stage host overhead of the GBDT stage loop, eager vs HIP-graph units:
125k rows per rank (an 8-GPU 1M-row job's shard) x 40 features, 100 stumps, on a one-rank
RCCL group (the per-stage all-reduce goes through RCCL) and without a group.  Prints host issue
time per stage (wall time of the loop's Python, no synchronisation) and device time per fit."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models import hist_gbdt  # noqa: E402
from hfens.models.gbdt import GradientBoostingClassifier  # noqa: E402
from hfens.models.hist_gbdt import fit_gbdt_batch  # noqa: E402

dev = torch.device("cuda", 0)
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000
T = 100
X, y = make_hf_cohort_device(rows, 40, seed=7, rows=(0, rows), device=dev)
import tempfile  # noqa: E402
store = tempfile.mktemp(prefix="hfens_pg_")
dist.init_process_group("nccl", init_method=f"file://{store}", rank=0, world_size=1, device_id=dev)
g = dist.new_group([0], backend="nccl")
res = {}
for name, group, mode in (("nogroup_eager", None, "0"), ("nogroup_graph", None, "1"),
                          ("rccl_eager", g, "0"), ("rccl_graph", g, "auto")):
    hist_gbdt.STAGE_GRAPH = mode
    host, wall = [], []
    for rep in range(6):
        ms = [GradientBoostingClassifier(n_estimators=T, max_depth=1, random_state=1)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fit_gbdt_batch(ms, X, y, group=group)
        torch.cuda.synchronize()
        if rep >= 2:
            wall.append(time.perf_counter() - t0)
            host.append(hist_gbdt.GRAPH_INFO["host_s"])
    res[name] = dict(host_us_per_stage=round(1e6 * sorted(host)[len(host) // 2] / (T + 2), 2),
                     fit_ms=round(1e3 * sorted(wall)[len(wall) // 2], 3),
                     units=hist_gbdt.GRAPH_INFO.get("units"),
                     per_stage_collectives=hist_gbdt.COLLECTIVES["per_stage"])
    print(name, res[name], flush=True)
dist.destroy_process_group()
print(json.dumps({"rows": rows, "trees": T, "results": res}))

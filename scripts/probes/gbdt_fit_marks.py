"""Host timeline (HFENS_TRACE_HOST marks, ms since the fit's start) of one GBDT fit at an 8-GPU
shard (125k rows) and at 1M rows, without a group and with a one-rank gloo group (the
data-parallel code paths: DP bin fit, peer reduction)."""
import os
import sys
import tempfile
import time

os.environ["HFENS_TRACE_HOST"] = "1"
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models.gbdt import GradientBoostingClassifier  # noqa: E402
from hfens.models.hist_gbdt import fit_gbdt_batch  # noqa: E402
from hfens.utils import timing  # noqa: E402

dev = torch.device("cuda", 0)
store = tempfile.mktemp(prefix="hfens_pg_")
dist.init_process_group("gloo", init_method=f"file://{store}", rank=0, world_size=1)
for rows in (125_000, 1_000_000):
    X, y = make_hf_cohort_device(rows, 40, seed=7, rows=(0, rows), device=dev)
    for name, group in (("nogroup", None), ("group1", dist.group.WORLD)):
        for rep in range(4):
            ms = [GradientBoostingClassifier(n_estimators=100, max_depth=1, random_state=1)]
            torch.cuda.synchronize()
            timing._MARKS.clear()
            t0 = time.perf_counter()
            fit_gbdt_batch(ms, X, y, group=group)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
        timing.hmarks_flush(f"[{rows} {name} wall {1e3 * wall:.2f} ms]")
from hfens.parallel import xgmi  # noqa: E402
xgmi.release_all()
dist.destroy_process_group()

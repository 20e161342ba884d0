"""Where a data-parallel GBDT fit spends its time (run under torchrun; ranks may share one GPU over
gloo): bin fit, tie-break ranks, stage loop, and the cost of one all-reduce of a stage slot."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.parallel import dist as pdist  # noqa: E402
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models.gbdt import GradientBoostingClassifier  # noqa: E402
from hfens.models import hist_gbdt  # noqa: E402
from hfens.models.binning import fit_bins  # noqa: E402

group, rank, world = pdist.init_from_env()
dev = pdist.rank_device()
torch.cuda.set_device(dev)
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
lo, hi = pdist.shard_bounds(rows, rank, world)
X, y = make_hf_cohort_device(rows, 40, seed=2020, rows=(lo, hi), device=dev)


def tm(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    dist.barrier(group)
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dist.barrier(group)
    return 1e3 * (time.perf_counter() - t) / reps


slot = torch.zeros(3 * 2112 + 8, dtype=torch.int64, device=dev)
t_ar = tm(lambda: dist.all_reduce(slot, group=group), reps=20)
t_bins = tm(lambda: fit_bins(X, 256, group))


def fit():
    m = [GradientBoostingClassifier(n_estimators=100, max_depth=1, random_state=1)]
    hist_gbdt.fit_gbdt_batch(m, X, y, group=group)


t_fit = tm(fit, reps=2)
if rank == 0:
    print(f"world {world} rows {rows}: one stage-slot all-reduce {t_ar:.2f} ms, bin fit {t_bins:.1f} ms, "
          f"full fit {t_fit:.1f} ms, path {hist_gbdt.LAST_PATH}", flush=True)
pdist.shutdown()

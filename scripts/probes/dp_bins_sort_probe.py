"""Cost of the pieces of the data-parallel bin fit on the device (run under torchrun)."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.parallel import dist as pdist  # noqa: E402
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models.binning import fit_bins  # noqa: E402

group, rank, world = pdist.init_from_env()
dev = pdist.rank_device()
torch.cuda.set_device(dev)
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
lo, hi = pdist.shard_bounds(rows, rank, world)
X, y = make_hf_cohort_device(rows, 40, seed=2020, rows=(lo, hi), device=dev)
X32 = X.to(torch.float32)


def tm(name, fn, reps=2):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    if rank == 0:
        print(f"{name}: {1e3 * (time.perf_counter() - t) / reps:.1f} ms", flush=True)


tm("segmented sort [F, n] dim=1", lambda: torch.sort((X32 + 0.0).t().contiguous(), dim=1))
Xt = X32.t().contiguous()
tm("F one-dimensional sorts", lambda: [torch.sort(Xt[f]) for f in range(Xt.shape[0])])
dist.barrier(group)
tm("fit_bins DP", lambda: fit_bins(X, 256, group), reps=1)
pdist.shutdown()

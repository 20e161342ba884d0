"""Time DP binning (order-statistic bisection) against the round-1 per-feature value-table
all-gathers, gloo on the CPU: python scripts/dp_bins_probe.py [world] [rows_per_rank] [F]."""
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _w(rank, world, port, n, F):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hfens.models import binning
    g = torch.Generator().manual_seed(rank)
    X = torch.randn(n, F, generator=g, dtype=torch.float64)
    X[:, : F // 4] = torch.randint(0, 3, (n, F // 4), generator=g).double()
    res = {}
    for mode in ("new", "legacy"):
        binning.LEGACY_DP_BINS = mode == "legacy"
        dist.barrier()
        t = time.perf_counter()
        bm = binning.fit_bins(X, 256, group=dist.group.WORLD)
        dist.barrier()
        res[mode] = (time.perf_counter() - t, bm)
    if rank == 0:
        a, b = res["new"][1], res["legacy"][1]
        same = torch.equal(a.edges, b.edges) and torch.equal(a.lo_val, b.lo_val)
        print(f"world {world} rows/rank {n} F {F}: bisection {res['new'][0]*1e3:.1f} ms | "
              f"value-table all-gathers {res['legacy'][0]*1e3:.1f} ms | identical bins {same}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 125000
    F = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    mp.spawn(_w, args=(world, 29631, n, F), nprocs=world)

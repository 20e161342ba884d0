"""cProfile the 1M-row GBDT bench fit (BASELINE config 3-GBC): host-side hotspots around the stage loop."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models.gbdt import GradientBoostingClassifier  # noqa: E402
from hfens.models.hist_gbdt import fit_gbdt_batch  # noqa: E402

dev = torch.device("cuda")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
X, y = make_hf_cohort_device(n, 40, seed=2020, rows=(0, n), device=dev)


def fit():
    ms = [GradientBoostingClassifier(n_estimators=100, max_depth=1, random_state=k) for k in range(seeds)]
    fit_gbdt_batch(ms, X, y)


for _ in range(2):
    fit()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    fit()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)

"""In-kernel phase stamps of one gbdt_stump_stage launch (HFENS_GBDT_STAGE_PROF=t)."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("HFENS_GBDT_STAGE_PROF", "50")
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models import hist_gbdt  # noqa: E402
from hfens.models.gbdt import GradientBoostingClassifier  # noqa: E402
dev = torch.device("cuda")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
X, y = make_hf_cohort_device(n, 40, seed=2020, rows=(0, n), device=dev)
for _ in range(2):
    m = GradientBoostingClassifier(n_estimators=100, max_depth=1, random_state=1)
    hist_gbdt.fit_gbdt_batch([m], X, y)
st = hist_gbdt.LAST_STAGE_PROF["stamps"]
st = st[st[:, 3] > 0]
q = np.percentile(st[:, :4], [50, 90, 100], axis=0)
print("groups", len(st), "cycles (median / p90 / max) at: split done, first sub-tile rows done, hist done, flushed")
print(q.astype(int))

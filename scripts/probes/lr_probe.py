"""Headline fit with the base models one after another (HFENS_CONCURRENT_BASES=0): the L1-LR
stage time and iteration counts for the HFENS_LOGREG_MEMBERS setting of the environment."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import logreg_solver  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
for rep in range(3):
    tm = StageTimer(enabled=True, device=dev)
    res = develop(Xd, yd, Xs, ys, names, device=dev, evaluate=False, timer=tm)
torch.cuda.synchronize()
lg = res.model.estimators_[2]
print(f"members={os.environ.get('HFENS_LOGREG_MEMBERS', 'auto')} path={logreg_solver.LAST_PATH}",
      {k: round(v * 1e3, 2) for k, v in tm.times.items() if k.startswith(("fit_", "oof_"))},
      "n_iter(final lg)", lg.n_iter_.tolist() if hasattr(lg.n_iter_, "tolist") else lg.n_iter_)

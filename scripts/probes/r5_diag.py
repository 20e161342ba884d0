"""Round-5 diagnostic: develop() on the bench cohort under switch combinations; prints the held-out
AUROC and the AUROC of each out-of-fold meta column against the development labels."""
import itertools
import sys

sys.path.insert(0, ".")
import numpy as np
import torch

from hfens import pipeline
from hfens.io.synth import make_hf_cohort
from hfens.models import hist_gbdt, stack_trainer
from hfens.utils import metrics

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
Xd, yd, names = make_hf_cohort(n, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(n, 40, seed=2021, nan_frac=0.02)
args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
for plan, pre, bases, ranks in itertools.product((0, 1), (0, 1), (0, 1), (0, 1)):
    if pre and not plan:
        continue
    pipeline.PLAN_AHEAD = bool(plan)
    stack_trainer.PRELAUNCH_SVC = bool(pre)
    stack_trainer.DEVICE_BASES = bool(bases)
    hist_gbdt.DEVICE_RANKS = bool(ranks)
    r = pipeline.develop(*args, names, device=dev)
    m = r.model.oof_meta_
    cols = [metrics.roc_auc(args[1], m[:, c]) for c in range(m.shape[1])]
    print(f"plan={plan} pre={pre} bases={bases} ranks={ranks} auroc={r.scores['auroc']:.4f} "
          f"oof_auc={[round(float(c), 4) for c in cols]} used={stack_trainer.LAST_PRELAUNCH['used']} "
          f"meta_coef={r.model.final_estimator_.coef_.cpu().numpy().round(4).tolist()}", flush=True)

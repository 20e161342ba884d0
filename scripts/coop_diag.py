"""Cooperative vs one-workgroup exact SMO on the same problems: per-fit iteration counts and the
largest α / ρ differences (diagnoses a diverging pair sequence vs rounding-level differences)."""
import sys

import torch

sys.path.insert(0, ".")
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo  # noqa: E402
from hfens.models.svc import SVC  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
slice_ = int(sys.argv[2]) if len(sys.argv) > 2 else 384
X, y, _ = make_hf_cohort(rows, 17, seed=21, nan_frac=0.0)
X, y = torch.as_tensor(X), torch.as_tensor(y)
dev = torch.device("cuda")
Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).to(dev)
yd = y.to(dev)
Zs, ys = [Z[: rows * 4 // 5], Z], [yd[: rows * 4 // 5], yd]
res = {}
for coop in (False, True):
    smo.COOP = coop
    smo.COOP_MIN_SLICE = slice_
    svcs = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in Zs]
    smo.fit_svc_batch(svcs, Zs, ys)
    res[coop] = (svcs, dict(smo.LAST_SMO_INFO))
for f, (a, b) in enumerate(zip(res[False][0], res[True][0])):
    d = (a._dual_coef_ - b._dual_coef_).abs()
    print(f"fit {f}: iters {int(a.n_iter_)} vs {int(b.n_iter_)}  n_sv {a.support_.numel()} vs {b.support_.numel()}  "
          f"max|dcoef| {float(d.max()):.3e} (#diff {int((d > 0).sum())})  "
          f"rho {float(a._intercept_[0]):.17g} vs {float(b._intercept_[0]):.17g}", flush=True)
print("members", res[False][1], res[True][1])

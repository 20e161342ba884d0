"""Phase breakdown of the cooperative SMO on the bench's SVC workload (HFENS_PROFILE_COOP=1):
per-pair s_memtime ticks of member 0 of every problem, split into WSS step 2, member reduction,
exchange 2, pair update, gradient update, step-1 reduction and exchange 1."""
import os
import sys

os.environ["HFENS_PROFILE_COOP"] = "1"
sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo  # noqa: E402
from hfens.pipeline import develop  # noqa: E402

dev = torch.device("cuda")
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
Xd, yd, names = make_hf_cohort(rows, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(rows, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
for _ in range(2):
    develop(Xd, yd, Xs, ys, names, device=dev)
torch.cuda.synchronize()
ph = smo.LAST_SMO_PROF["phases"].astype(np.float64)
it = smo.LAST_SMO_PROF["iters"].astype(np.float64)
print("info", smo.LAST_SMO_INFO)
names_ph = ["step2", "red2", "xchg2", "pair", "update", "red1", "xchg1"]
k = int(np.argmax(ph.sum(1)))
print(f"slowest problem {k}: iters {int(it[k])}, total ticks {ph[k].sum():.0f}")
for n, v in zip(names_ph, ph[k]):
    print(f"  {n:7s} {v / max(it[k], 1):9.1f} ticks/pair  {100 * v / ph[k].sum():5.1f} %")

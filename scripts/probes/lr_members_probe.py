"""Device time of the fused logistic-regression launch vs members per model (the stacking meta
model: 10k rows × 3 meta-features + intercept, L2; and the 6-model L1 base fit at 10k × 17)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.models import logreg_solver  # noqa: E402
from hfens.models.linear import LogisticRegression  # noqa: E402
from hfens.models.logreg_solver import fit_logreg_batch  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
for (n, F, B, pen) in ((10000, 3, 1, "l2"), (10000, 17, 6, "l1"), (100000, 3, 1, "l2")):
    X = torch.randn(n, F, generator=g, dtype=torch.float64)
    w = torch.randn(F, generator=g, dtype=torch.float64)
    y = ((X @ w + 0.5 * torch.randn(n, generator=g, dtype=torch.float64)) > 0).double()
    X, y = X.to(dev), y.to(dev)
    masks = torch.ones(B, n, dtype=torch.bool, device=dev)
    for k in range(1, B):
        masks[k, k::B] = False
    for M in (1, 2, 4, 8, 16):
        logreg_solver.MEMBERS = M
        ts = []
        for rep in range(6):
            ms = [LogisticRegression(penalty=pen, solver="liblinear" if pen == "l1" else "lbfgs") for _ in range(B)]
            for m in ms:
                m.emulate_liblinear = False
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            fit_logreg_batch(ms, X, y, masks)
            e1.record()
            torch.cuda.synchronize()
            if rep >= 2:
                ts.append(e0.elapsed_time(e1))
        print(f"n={n} F={F} B={B} {pen} members={logreg_solver.LAST_PATH.get('members')}: "
              f"{sorted(ts)[1]:.3f} ms  iters={[int(m.n_iter_[0]) for m in ms][:3]}", flush=True)
logreg_solver.MEMBERS = 0

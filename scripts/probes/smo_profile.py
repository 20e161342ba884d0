"""Per-problem SMO iteration counts and batch time for the 10k x 17 stacking SVC fits."""
import sys, time, numpy as np, torch
sys.path.insert(0, '.')
from hfens.io.synth import make_hf_cohort
from hfens.models import smo
from hfens.models.svc import SVC
from hfens.models.model_selection import stratified_kfold_test_folds, fold_masks
dev = torch.device('cuda')
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
X, y, _ = make_hf_cohort(n, 17, seed=3, nan_frac=0.0)
X = torch.as_tensor(X, device=dev); y = torch.as_tensor(y, device=dev)
masks = fold_masks(stratified_kfold_test_folds(y.cpu().numpy(), 5), 5, device=dev)
Zs, ys, svcs = [], [], []
for m in masks:
    r = torch.nonzero(m).squeeze(1); Xm = X[r]
    Zs.append((Xm - Xm.mean(0)) / Xm.std(0, unbiased=False)); ys.append(y[r])
    svcs.append(SVC(class_weight='balanced', probability=True, random_state=2020))
probs, meta = [], []
for f, (s, Z, yy) in enumerate(zip(svcs, Zs, ys)):
    pr, mt = smo._expand(f, Z, yy, s, dev); probs += pr
for rep in range(2):
    torch.cuda.synchronize(); t = time.perf_counter()
    sol = smo._solve_device(probs, Zs, dev, 1e-3)
    torch.cuda.synchronize(); dt = time.perf_counter() - t
    its = [int(sol[id(p)][2]) for p in probs if p.rows is not None]
    ls = [int(p.rows.numel()) for p in probs if p.rows is not None]
    print(f"rep {rep}: solve {dt*1e3:.1f} ms  max_iter {max(its)}  iters {its[:6]}  l {ls[:6]}")
print("us/iter (max problem)", dt * 1e6 / max(its))

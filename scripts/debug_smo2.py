import sys, numpy as np, torch
sys.path.insert(0, '.')
from hfens.io.synth import make_hf_cohort
from hfens.models.svc import SVC
X, y, _ = make_hf_cohort(1500, 17, seed=14, nan_frac=0)
X = torch.as_tensor(X); y = torch.as_tensor(y)
Z = (X - X.mean(0)) / X.std(0, unbiased=False)
dev = torch.device('cuda')
for prob in (False, True):
    mh = SVC(class_weight="balanced", probability=prob, random_state=2020).fit(Z, y)
    md = SVC(class_weight="balanced", probability=prob, random_state=2020).fit(Z.to(dev), y.to(dev))
    print('prob', prob, 'nsv', mh._n_support.tolist(), md._n_support.cpu().tolist(), 'rho', mh._intercept_.item(), md._intercept_.item())
    print(' coef maxdiff', float((mh._dual_coef_ - md._dual_coef_.cpu()).abs().max()) if mh._dual_coef_.shape == md._dual_coef_.shape else 'shape', 'A,B', mh._probA.item(), md._probA.item(), mh._probB.item(), md._probB.item())
    dh = mh.decision_function(Z); dd = md.decision_function(Z.to(dev)).cpu()
    dd2 = md.to('cpu').decision_function(Z)
    print(' dec host-vs-dev', float((dh - dd).abs().max()), 'dev-model-on-cpu', float((dh - dd2).abs().max()))

import sys, numpy as np, torch
sys.path.insert(0, '.')
from hfens.io.synth import make_hf_cohort
from hfens.models.svc import SVC
from sklearn.preprocessing import StandardScaler
from sklearn.svm import SVC as SK
X, y, _ = make_hf_cohort(1500, 17, seed=14, nan_frac=0)
Z = StandardScaler().fit_transform(X)
sk = SK(class_weight="balanced", probability=True, random_state=2020).fit(Z, y)
dev = torch.device('cuda')
Zt = torch.as_tensor(Z)
for rep in range(3):
    m = SVC(class_weight="balanced", probability=True, random_state=2020)
    m.fit(Zt.to(dev), torch.as_tensor(y).to(dev))
    d = m.decision_function(Zt.to(dev)).cpu().numpy()
    print(rep, 'nsv', m._n_support.cpu().tolist(), sk.n_support_, 'rho', m._intercept_.item(), sk._intercept_, 'dec diff', np.abs(d - sk.decision_function(Z)).max(), m.n_iter_)
mh = SVC(class_weight="balanced", probability=True, random_state=2020).fit(Zt, torch.as_tensor(y))
print('host', mh._n_support.tolist(), np.abs(mh.decision_function(Zt).numpy() - sk.decision_function(Z)).max())

import sys, numpy as np, torch
sys.path.insert(0, '.')
from hfens.io.synth import make_hf_cohort
from hfens.models import smo
X, y, _ = make_hf_cohort(1500, 17, seed=14, nan_frac=0)
X = torch.as_tensor(X); y = torch.as_tensor(y)
Z = (X - X.mean(0)) / X.std(0, unbiased=False)
from hfens.models.svc import SVC
svc = SVC(class_weight="balanced", probability=False, random_state=2020)
probs, mt = smo._expand(0, Z, y, svc, 'cpu')
p = probs[-1]
dev = torch.device('cuda')
Zd = Z.to(dev)
pd = smo._Prob(0, -1, p.rows.to(dev), p.npos, p.Cp, p.Cn, p.gamma)
out = smo._solve_device([pd], [Zd], dev, 1e-3)
a, r, it = out[id(pd)]
print('device iters', int(it), 'rho', float(r), 'nsv', int((a > 0).sum()))
hout = smo._solve_host([p], [Z], 1e-3)
ah, rh, ith = hout[id(p)]
print('host iters', int(ith), 'rho', float(rh), 'nsv', int((ah > 0).sum()))
print('alpha maxdiff', float((a.cpu() - ah).abs().max()))
# check gram
from hfens.models.smo import _gram_host
Kh = _gram_host(Z[p.rows].double().numpy(), p.gamma)
import hfens.ops as ops
E = ops.ext()
l = p.rows.numel(); ld = (l + 63) // 64 * 64
g = np.zeros(1, smo._GRAM_DT); g[0] = (0, 0, l, ld, -p.gamma * 1.4426950408889634, 0)
K = torch.empty(l * ld, dtype=torch.float32, device=dev)
zc = Zd[pd.rows].float().contiguous()
E.gram_rbf_batch(zc.data_ptr(), 17, smo._dev_struct(g, dev).data_ptr(), 1, l, K.data_ptr(), ops.stream_ptr(dev))
Kd = K.view(l, ld)[:, :l].cpu().numpy()
print('gram maxdiff', np.abs(Kd - Kh).max(), 'diag', Kd.diagonal()[:3])

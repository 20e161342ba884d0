"""Training kernels on the MI355X vs the host mirrors / installed sklearn."""
import numpy as np
import pytest
import torch

from hfens.io.synth import make_hf_cohort
from hfens.models.gbdt import GradientBoostingClassifier
from hfens.models.hist_gbdt import fit_gbdt_batch
from hfens.models.linear import LogisticRegression
from hfens.models.logreg_solver import fit_logreg_batch
from hfens.models.svc import SVC

pytestmark = pytest.mark.gpu


def _data(n, F, seed, nan=0.0):
    X, y, _ = make_hf_cohort(n, F, seed=seed, nan_frac=nan)
    return torch.as_tensor(X), torch.as_tensor(y)


@pytest.mark.parametrize("depth", [1, 3])
def test_gbdt_device_matches_host(dev, depth):
    X, y = _data(3000, 40, 11)
    masks = torch.ones(3, 3000, dtype=torch.bool)
    masks[0, :1000] = False
    masks[1, 1000:2000] = False
    mh = [GradientBoostingClassifier(n_estimators=20, max_depth=depth) for _ in range(3)]
    md = [GradientBoostingClassifier(n_estimators=20, max_depth=depth) for _ in range(3)]
    fit_gbdt_batch(mh, X, y, masks)
    fit_gbdt_batch(md, X.to(dev), y.to(dev), masks.to(dev))
    for a, b in zip(mh, md):
        assert torch.equal(a.tree_feature_, b.tree_feature_.cpu())
        assert torch.allclose(a.tree_value_, b.tree_value_.cpu(), rtol=1e-9, atol=1e-12)
        assert torch.allclose(a.train_score_, b.train_score_.cpu(), rtol=1e-9)
        pa = a.predict_proba(X)[:, 1]
        pb = b.predict_proba(X.to(dev))[:, 1].cpu()
        assert torch.allclose(pa, pb, atol=2e-6)


def test_gbdt_vs_sklearn_stumps(dev):
    from sklearn.ensemble import GradientBoostingClassifier as SK
    X, y = _data(2000, 17, 12)
    m = GradientBoostingClassifier(n_estimators=100, max_depth=1)
    fit_gbdt_batch([m], X.to(dev), y.to(dev))
    sk = SK(n_estimators=100, max_depth=1, random_state=0).fit(X.numpy(), y.numpy())
    p = m.predict_proba(X.to(dev))[:, 1].cpu().numpy()
    assert np.abs(p - sk.predict_proba(X.numpy())[:, 1]).max() < 1e-5
    assert np.abs(m.train_score_.cpu().numpy() - sk.train_score_).max() < 1e-6


@pytest.mark.parametrize("pen", ["l1", "l2"])
def test_logreg_device_matches_host(dev, pen):
    X, y = _data(4000, 40, 13)
    masks = torch.ones(2, 4000, dtype=torch.bool)
    masks[0, ::3] = False
    kw = dict(penalty=pen, solver="liblinear" if pen == "l1" else "lbfgs", class_weight="balanced")
    mh = [LogisticRegression(**kw) for _ in range(2)]
    md = [LogisticRegression(**kw) for _ in range(2)]
    fit_logreg_batch(mh, X, y, masks)
    fit_logreg_batch(md, X.to(dev), y.to(dev), masks.to(dev))
    for a, b in zip(mh, md):
        assert torch.allclose(a.coef_, b.coef_.cpu(), atol=1e-6)


def test_svc_device_matches_libsvm(dev):
    from sklearn.preprocessing import StandardScaler
    from sklearn.svm import SVC as SK
    X, y = _data(1500, 17, 14)
    Z = StandardScaler().fit_transform(X.numpy())
    sk = SK(class_weight="balanced", probability=True, random_state=2020).fit(Z, y.numpy())
    m = SVC(class_weight="balanced", probability=True, random_state=2020)
    m.fit(torch.as_tensor(Z).to(dev), y.to(dev))
    d = m.decision_function(torch.as_tensor(Z).to(dev)).cpu().numpy()
    assert np.abs(d - sk.decision_function(Z)).max() < 5e-3
    p = m.predict_proba(torch.as_tensor(Z).to(dev))[:, 1].cpu().numpy()
    assert np.abs(p - sk.predict_proba(Z)[:, 1]).max() < 5e-3
    assert abs(int(m._n_support.sum()) - int(sk.n_support_.sum())) <= 0.02 * len(Z)


def test_svc_device_matches_host_exactly(dev):
    X, y = _data(600, 17, 15)
    Z = (X - X.mean(0)) / X.std(0, unbiased=False)
    mh = SVC(class_weight="balanced", probability=True, random_state=2020).fit(Z, y)
    md = SVC(class_weight="balanced", probability=True, random_state=2020).fit(Z.to(dev), y.to(dev))
    assert torch.equal(mh.support_.cpu(), md.support_.cpu())
    assert abs(float(mh._intercept_[0]) - float(md._intercept_[0])) < 1e-4
    assert abs(mh._probA.item() - md._probA.item()) < 1e-3


def test_gbdt_subsample_device_matches_host(dev):
    X, y = _data(3000, 20, 31)
    mh = [GradientBoostingClassifier(n_estimators=20, max_depth=2, subsample=0.7, random_state=s) for s in (3, 4)]
    md = [GradientBoostingClassifier(n_estimators=20, max_depth=2, subsample=0.7, random_state=s) for s in (3, 4)]
    fit_gbdt_batch(mh, X, y)
    fit_gbdt_batch(md, X.to(dev), y.to(dev))
    for a, b in zip(mh, md):
        assert torch.equal(a.tree_feature_, b.tree_feature_.cpu())
        assert torch.allclose(a.tree_value_, b.tree_value_.cpu(), rtol=1e-9, atol=1e-12)
        assert torch.allclose(a.train_score_, b.train_score_.cpu(), rtol=1e-9)


def test_binned_stump_tables_match_tree_walk(dev):
    from hfens.models.forest_infer import ensemble_raw_binned, stump_bin_tables
    X, y = _data(5003, 24, 41)
    ms = [GradientBoostingClassifier(n_estimators=60, max_depth=1, subsample=0.8, random_state=s) for s in (1, 2, 3)]
    fit_gbdt_batch(ms, X.to(dev), y.to(dev))
    T, init = stump_bin_tables(ms)
    bins = ms[0]._bin_mapper.transform(X.to(dev))
    got = ensemble_raw_binned(T, init, bins).double().cpu()
    ref = ensemble_raw_binned(T.cpu(), init.cpu(), bins.cpu())
    assert torch.allclose(got, ref, atol=2e-5)
    for b, m in enumerate(ms):
        walk = m.decision_function(X.to(dev)).cpu()
        assert torch.allclose(got[b], walk, atol=2e-5)

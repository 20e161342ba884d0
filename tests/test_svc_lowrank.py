"""Large-problem SVC (Nyström reduced set + interior-point dual, hfens/models/svc_lowrank.py)."""
import numpy as np
import torch

from hfens.io.synth import make_hf_cohort


def _data(n, seed):
    X, y, _ = make_hf_cohort(n, 12, seed=seed, nan_frac=0.0)
    return np.asarray(X), np.asarray(y)


def test_full_rank_equals_libsvm():
    """landmarks = every row ⇒ K̃ = K: the IPM optimum is libsvm's to its own 1e-3 tolerance."""
    from sklearn.svm import SVC as SkSVC
    from hfens.models.svc import SVC
    from hfens.models.svc_lowrank import fit_svc_lowrank_batch
    X, y = _data(500, 41)
    mu, sd = X.mean(0), X.std(0)
    Z = (X - mu) / sd
    Xt, _ = _data(400, 42)
    Zt = (Xt - mu) / sd
    ours = SVC(class_weight="balanced", probability=True, random_state=2020)
    fit_svc_lowrank_batch([ours], [torch.as_tensor(Z)], [torch.as_tensor(y)], n_landmarks=500)
    ref = SkSVC(class_weight="balanced", probability=True, random_state=2020).fit(Z, y)
    d = ours.decision_function(torch.as_tensor(Zt)).numpy()
    assert np.abs(d - ref.decision_function(Zt)).max() < 5e-3   # libsvm stops at a 1e-3 KKT gap
    p = ours.predict_proba(torch.as_tensor(Zt)).numpy()[:, 1]
    assert np.abs(p - ref.predict_proba(Zt)[:, 1]).max() < 2e-3


def test_ipm_matches_smo_on_lowrank_kernel():
    """Same QP, two solvers: the IPM optimum vs libsvm's SMO (host mirror, eps 1e-7) on the
    explicit low-rank Gram ΦΦᵀ — equal dual objectives, equal decision values, equal ρ."""
    from hfens.models.smo import _smo_host
    from hfens.models.svc_lowrank import ipm_svc_dual, nystrom_map
    X, y = _data(600, 43)
    Z = torch.as_tensor((X - X.mean(0)) / X.std(0))
    order = np.argsort(y > 0.5, kind="stable")          # +1 (class 0) first, as _smo_host expects
    Z = Z[torch.as_tensor(order)]
    yy = torch.as_tensor(np.where(y[order] > 0.5, -1.0, 1.0))
    npos = int((yy > 0).sum())
    Phi, _ = nystrom_map(Z, torch.arange(0, 600, 3), 1 / 12)
    c = torch.where(yy > 0, 0.6, 2.7).double()
    a, rho, it = ipm_svc_dual(Phi, yy, c)
    assert it < 60
    assert bool((a >= 0).all()) and bool((a <= c).all())
    assert abs(float(torch.dot(yy, a))) < 1e-6 * float(c.sum())
    K = (Phi @ Phi.T).numpy()
    a2, rho2, _ = _smo_host(K, npos, 0.6, 2.7, 1e-7, 10_000_000)
    a2 = torch.as_tensor(a2)

    def obj(al):
        v = yy * al
        return 0.5 * float(v @ (Phi @ (Phi.T @ v))) - float(al.sum())
    assert abs(obj(a) - obj(a2)) < 1e-6 * abs(obj(a2))
    dec = Phi @ (Phi.T @ (yy * a)) - rho
    dec2 = Phi @ (Phi.T @ (yy * a2)) - rho2
    assert float((dec - dec2).abs().max()) < 1e-4
    assert abs(rho - rho2) < 1e-5


def test_auto_switch_and_auroc_vs_exact():
    """Forced low-rank on a stack fit: same held-out AUROC as the exact solver within 0.01."""
    from hfens.io.synth import make_dev_select
    from hfens.models import smo
    from hfens.pipeline import develop
    Xd, yd, Xs, ys, names = make_dev_select(700, 30, seed=44)
    assert smo.use_lowrank([40000]) and not smo.use_lowrank([10000])
    exact = develop(Xd, yd, Xs, ys, names, device="cpu")
    old = smo.SOLVER
    smo.SOLVER = "lowrank"
    try:
        low = develop(Xd, yd, Xs, ys, names, device="cpu")
    finally:
        smo.SOLVER = old
    assert smo.LAST_SMO_INFO["solver"] == "nystrom-ipm"
    assert abs(low.scores["auroc"] - exact.scores["auroc"]) < 0.01

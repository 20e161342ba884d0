"""Preprocessing kernels on the MI355X: KNN donor search and the LassoCV path vs host mirrors."""
import numpy as np
import pytest
import torch

from hfens.io.synth import make_hf_cohort
from hfens.models.imputer import KNNImputer
from hfens.models.lasso import LassoCV, SelectFromModel
from hfens import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mfma", ["auto", "1"])
@pytest.mark.parametrize("n,F,nan", [(3000, 40, 0.02), (700, 64, 0.05), (500, 17, 0.3), (6000, 40, 0.05)])
def test_knn_imputer_device_matches_host(dev, monkeypatch, n, F, nan, mfma):
    """The device imputation equals the host f64 mirror bit for bit — with the packed-FMA search
    and with the matrix-core filter forced (its donor search AND its f64-refine window listing)."""
    from hfens.models import imputer as imp_mod
    monkeypatch.setattr(imp_mod, "MFMA_FILTER", mfma)
    X, _, _ = make_hf_cohort(n, F, seed=n + F, nan_frac=nan)
    X = np.concatenate([X, X[: n // 20] + 1e-9 * (n % 7)], axis=0)   # near-duplicate donors: f32 near-ties
    Xt = torch.as_tensor(X)
    host = KNNImputer(n_neighbors=1).fit(Xt).transform(Xt)
    devo = KNNImputer(n_neighbors=1).fit(Xt.to(dev)).transform(Xt.to(dev)).cpu()
    # f32 search + f64 refine of its near-ties (knn.hip knn_refine): the host mirror's f64 donors
    assert torch.equal(host, devo), int(((host - devo).abs() > 0).sum())


def test_knn_matches_sklearn(dev):
    from sklearn.impute import KNNImputer as SK
    X, _, _ = make_hf_cohort(2000, 40, seed=9, nan_frac=0.02)
    ours = KNNImputer(n_neighbors=1).fit(torch.as_tensor(X).to(dev)).transform(torch.as_tensor(X).to(dev)).cpu().numpy()
    theirs = SK(n_neighbors=1).fit_transform(X)
    assert (np.abs(ours - theirs) > 1e-9).sum() <= max(1, int(0.01 * np.isnan(X).sum()))


def test_lasso_device_matches_host(dev):
    X, y, _ = make_hf_cohort(4000, 40, seed=21, nan_frac=0.0)
    Xt, yt = torch.as_tensor(X), torch.as_tensor(y)
    h = SelectFromModel(LassoCV(cv=10), threshold=-np.inf, max_features=17).fit(Xt, yt)
    d = SelectFromModel(LassoCV(cv=10), threshold=-np.inf, max_features=17).fit(Xt.to(dev), yt.to(dev))
    assert abs(h.estimator_.alpha_ - d.estimator_.alpha_) < 1e-12
    assert np.array_equal(h.get_support(), d.get_support())
    assert torch.allclose(h.estimator_.coef_, d.estimator_.coef_.cpu(), atol=1e-9)


def test_weighted_moments(dev):
    g = torch.Generator().manual_seed(0)
    X = torch.randn(5000, 41, generator=g, dtype=torch.float64)
    W = torch.rand(7, 5000, generator=g, dtype=torch.float64)
    V = torch.randn(7, 5000, generator=g, dtype=torch.float64)
    G, a, v = ops.weighted_moments(X.to(dev), W.to(dev), V.to(dev))
    Gr, ar, vr = ops.weighted_moments(X, W, V)
    assert torch.allclose(G.cpu(), Gr, rtol=1e-12, atol=1e-9)
    assert torch.allclose(a.cpu(), ar, rtol=1e-12, atol=1e-9)
    assert torch.allclose(v.cpu(), vr, rtol=1e-12, atol=1e-9)


def test_lasso_speculative_refit_bit_identical(dev, monkeypatch):
    """The all-alpha cold-start refits solved on a side stream beside the CV paths (the winner picked
    afterwards) give exactly the one-problem refit at the chosen alpha."""
    from hfens.models import lasso
    X, y, _ = make_hf_cohort(5000, 40, seed=9, nan_frac=0.0)
    Xt, yt = torch.as_tensor(X, device=dev), torch.as_tensor(y, device=dev)
    out = {}
    for spec in (False, True):
        monkeypatch.setattr(lasso, "SPECULATIVE_REFIT", spec)
        m = LassoCV(cv=10).fit(Xt, yt)
        out[spec] = (m.alpha_, m.coef_.cpu(), float(m.intercept_))
    assert out[False][0] == out[True][0]
    assert torch.equal(out[False][1], out[True][1])
    assert out[False][2] == out[True][2]


@pytest.mark.parametrize("idx", [-1, 0])
def test_lasso_early_speculation_bit_identical(dev, monkeypatch, idx):
    """The early speculation (lasso.EARLY_SPEC: the speculated grid point computed on the device,
    its refit enqueued before the grid's host read, no every-alpha refit) gives exactly the
    non-speculative fit — α, coefficients, intercept, selection — when it hits (idx −1, the
    smallest alpha: the cohort's winner) and when it misses (idx 0: the one refit after the paths);
    its device alpha equals the host grid's end point bit for bit, and the early overlap runs
    before the late one."""
    from hfens.models import lasso
    X, y, _ = make_hf_cohort(5000, 40, seed=9, nan_frac=0.0)
    Xt, yt = torch.as_tensor(X, device=dev), torch.as_tensor(y, device=dev)
    out = {}
    for spec in (False, True):
        monkeypatch.setattr(lasso, "SPECULATE", spec)
        monkeypatch.setattr(lasso, "SPEC_ALPHA_INDEX", idx)
        order = []
        s = lasso.SelectFromModel(LassoCV(cv=10), threshold=-np.inf, max_features=17)
        s.fit(Xt, yt, overlap=lambda: order.append("late"), early_overlap=lambda: order.append("early"))
        m = s.estimator_
        assert order == ["early", "late"]
        out[spec] = (m.alpha_, m.coef_.cpu(), float(m.intercept_), s.get_support().copy(),
                     s.cols_dev_.cpu().numpy())
        if spec:
            assert float(m.spec_alpha_dev_) == float(m.alphas_[idx])
            assert bool(s.cols_speculative_)
    assert out[False][0] == out[True][0]
    assert torch.equal(out[False][1], out[True][1])
    assert out[False][2] == out[True][2]
    assert np.array_equal(out[False][3], out[True][3])
    assert np.array_equal(out[False][4], np.nonzero(out[False][3])[0])
    assert np.array_equal(out[True][4], np.nonzero(out[True][3])[0]) == (idx == -1)


@pytest.mark.parametrize("n,F,nan", [(20000, 40, 0.02), (6000, 17, 0.1), (3000, 64, 0.3), (4000, 33, 0.0)])
def test_knn_fast_pass_same_donors(dev, monkeypatch, n, F, nan):
    """the packed-FMA fast pass with its exact lower-bound skip
    (knn_donor_fast_kernel, default) picks the SAME donors as the exact masked direct-difference
    kernel for every missing cell (HFENS_KNN_KERNEL=direct): identical imputed matrices, exact ties
    (binary features, duplicated rows) included."""
    X, _, _ = make_hf_cohort(n, F, seed=3 * n + F, nan_frac=nan)
    X = np.concatenate([X, X[: n // 10]], axis=0)            # duplicated rows: exact distance ties
    if nan == 0.0:
        X[::7, 3] = np.nan                                   # a few receivers still
    Xt = torch.as_tensor(X, device=dev)
    out = {}
    for k in ("direct", "fast"):
        monkeypatch.setenv("HFENS_KNN_KERNEL", k)
        imp = KNNImputer(n_neighbors=1).fit(Xt)
        out[k] = imp.transform(Xt).cpu()
    assert torch.equal(out["direct"], out["fast"])


@pytest.mark.parametrize("n,F,nan", [(3000, 40, 0.02), (2500, 17, 0.1), (2000, 24, 0.3), (1500, 48, 0.05),
                                     (60000, 40, 0.02)])
def test_knn_mfma_filter_same_slots(dev, n, F, nan):
    """the donor search with its filter on the bf16 matrix cores
    (knn.hip knn_donor_mfma_kernel) gives the SAME per-slot best (f32 distance bits, donor) and the
    same runner-up distances as the packed-FMA kernel — the exact pass decides both, the matrix-core
    bound only skips donors that cannot matter — duplicated rows (exact ties) included."""
    from hfens import ops
    X, _, _ = make_hf_cohort(n, F, seed=7 * n + F, nan_frac=nan)
    X = np.concatenate([X, X[: n // 10]], axis=0)
    X[::11, 2] = np.nan
    mu = np.nanmean(X, 0)
    miss = np.isnan(X)
    Xc = np.where(miss, 0.0, X - mu).astype(np.float32)
    bits = (miss.astype(np.uint64) << np.arange(F, dtype=np.uint64)).sum(1).astype(np.uint64).view(np.int64)
    rows = np.nonzero(miss.any(1))[0]
    slot = np.full((rows.shape[0], 8), -1, dtype=np.int32)
    for i, r in enumerate(rows):
        c = np.nonzero(miss[r])[0][:8]
        slot[i, :c.shape[0]] = c
    E = ops.ext()
    s = ops.stream_ptr(dev)
    R = torch.as_tensor(Xc[rows], device=dev).contiguous()
    rm = torch.as_tensor(bits[rows], device=dev)
    D = torch.as_tensor(Xc, device=dev).contiguous()
    dm = torch.as_tensor(bits, device=dev)
    sl = torch.as_tensor(slot, device=dev)
    nr, nd = R.shape[0], D.shape[0]
    out = {}
    for kind in ("fast", "mfma"):
        best = torch.empty(nr, 8, dtype=torch.int64, device=dev)
        alt = torch.empty(nr, 8, dtype=torch.int32, device=dev)
        if kind == "fast":
            E.knn_donors(R.data_ptr(), rm.data_ptr(), nr, D.data_ptr(), dm.data_ptr(), nd, F, sl.data_ptr(),
                         best.data_ptr(), alt.data_ptr(), 0, 0, s)
        else:
            wd = np.zeros(1, dtype=np.int64)
            E.knn_mfma_item_words(F, wd.ctypes.data)
            items = torch.empty(nd * int(wd[0]), dtype=torch.int32, device=dev)
            ny = torch.empty(nd, dtype=torch.float32, device=dev)
            E.knn_mfma_prep(D.data_ptr(), dm.data_ptr(), nd, F, items.data_ptr(), ny.data_ptr(), s)
            E.knn_donors_mfma(R.data_ptr(), rm.data_ptr(), nr, D.data_ptr(), dm.data_ptr(), nd, F, sl.data_ptr(),
                              best.data_ptr(), alt.data_ptr(), 0, 0, items.data_ptr(), ny.data_ptr(), s)
        torch.cuda.synchronize()
        out[kind] = (best.cpu(), alt.cpu())
    assert torch.equal(out["fast"][0], out["mfma"][0])
    assert torch.equal(out["fast"][1], out["mfma"][1])


def test_knn_imputer_mfma_same_output(dev, monkeypatch):
    """The imputer's output with the matrix-core donor filter forced on equals the packed-FMA path's
    bit for bit (the exact passes decide the donors; f64 refine and apply are shared)."""
    from hfens.models import imputer as imp_mod
    from hfens.models.imputer import KNNImputer
    X, _, _ = make_hf_cohort(20000, 40, seed=5, nan_frac=0.03)
    X = np.concatenate([X, X[:1500] + 1e-9], axis=0)   # near-duplicate donors: the f64 refine's windows
    Xt = torch.as_tensor(X, device=dev)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(imp_mod, "MFMA_FILTER", mode)
        out[mode] = KNNImputer(n_neighbors=1).fit(Xt).transform(Xt).cpu()
    assert not torch.isnan(out["1"]).any()
    assert torch.equal(out["0"], out["1"])

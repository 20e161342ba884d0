"""End-to-end development flow vs the reference pipeline re-run with the installed
scikit-learn (reference train_ensemble_public.py:37-64, plots omitted)."""
import numpy as np
import pytest
import torch

from hfens.io.synth import make_dev_select
from hfens.pipeline import develop


def _sklearn_reference(Xd, yd, Xs, ys):
    from sklearn.ensemble import GradientBoostingClassifier, StackingClassifier
    from sklearn.feature_selection import SelectFromModel
    from sklearn.impute import KNNImputer
    from sklearn.linear_model import LassoCV, LogisticRegression
    from sklearn.pipeline import make_pipeline
    from sklearn.preprocessing import StandardScaler
    from sklearn.svm import SVC
    from sklearn.metrics import roc_auc_score
    np.random.seed(2020)
    imp = KNNImputer(missing_values=np.nan, n_neighbors=1)
    Xd = imp.fit_transform(Xd)
    Xs = imp.transform(Xs)
    est = [("svc", make_pipeline(StandardScaler(), SVC(class_weight="balanced", probability=True, random_state=2020))),
           ("gbc", GradientBoostingClassifier(n_estimators=100, max_depth=1, random_state=2020)),
           ("lg", LogisticRegression(class_weight="balanced", penalty="l1", solver="liblinear"))]
    clf = StackingClassifier(estimators=est, final_estimator=LogisticRegression(class_weight="balanced"))
    sfm = SelectFromModel(LassoCV(random_state=2020, cv=10), threshold=-np.inf, max_features=17).fit(Xd, yd)
    m = sfm.get_support()
    clf.fit(Xd[:, m], yd)
    p = clf.predict_proba(Xs[:, m])[:, 1]
    return m, p, roc_auc_score(ys, p)


@pytest.mark.slow
def test_develop_matches_sklearn_pipeline():
    Xd, yd, Xs, ys, names = make_dev_select(713, 64, seed=2020)
    res = develop(Xd, yd, Xs, ys, names, device="cpu")
    m, p, auc = _sklearn_reference(Xd.copy(), yd, Xs.copy(), ys)
    assert np.array_equal(res.selected, m)
    ours = res.proba_sel.numpy()
    # same selected features; stack probabilities agree to the solvers' tolerances
    assert np.abs(ours - p).max() < 0.02
    assert abs(res.scores["auroc"] - auc) < 0.005


def test_classification_report_format():
    from sklearn.metrics import classification_report as skr
    from hfens.utils.metrics import classification_report
    rng = np.random.default_rng(0)
    y = (rng.random(300) < 0.2).astype(float)
    p = rng.random(300) > 0.6
    assert classification_report(torch.as_tensor(y), torch.as_tensor(p.astype(float))) == skr(y, p)


def test_auc_ap_match_sklearn():
    from sklearn.metrics import average_precision_score, roc_auc_score, roc_curve as skroc
    from hfens.utils import metrics
    rng = np.random.default_rng(1)
    y = (rng.random(2000) < 0.25).astype(float)
    s = np.round(rng.random(2000) + 0.3 * y, 2)  # ties
    assert abs(metrics.roc_auc(torch.as_tensor(y), torch.as_tensor(s)) - roc_auc_score(y, s)) < 1e-12
    assert abs(metrics.average_precision(torch.as_tensor(y), torch.as_tensor(s)) - average_precision_score(y, s)) < 1e-12
    fpr, tpr, _ = metrics.roc_curve(torch.as_tensor(y), torch.as_tensor(s))
    f2, t2, _ = skroc(y, s)
    np.testing.assert_allclose(fpr.numpy(), f2)
    np.testing.assert_allclose(tpr.numpy(), t2)


def test_binned_stump_tables_host():
    from hfens.io.synth import make_hf_cohort
    from hfens.models.forest_infer import ensemble_raw_binned, stump_bin_tables
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.models.hist_gbdt import fit_gbdt_batch
    X, y, _ = make_hf_cohort(800, 12, seed=4, nan_frac=0.0)
    X, y = torch.as_tensor(X), torch.as_tensor(y)
    ms = [GradientBoostingClassifier(n_estimators=30, max_depth=1, random_state=s) for s in (1, 2)]
    fit_gbdt_batch(ms, X, y)
    T, init = stump_bin_tables(ms)
    raw = ensemble_raw_binned(T, init, ms[0]._bin_mapper.transform(X))
    for b, m in enumerate(ms):
        assert torch.allclose(raw[b], m.decision_function(X), atol=1e-9)


def test_save_plots_png_and_svg_fallback(tmp_path, monkeypatch):
    from hfens.utils import metrics
    y = torch.tensor([0, 1, 0, 1, 1, 0, 0, 1.0])
    p = torch.tensor([.1, .9, .3, .6, .8, .2, .55, .4])
    out = metrics.save_plots(y, p, str(tmp_path / "a"))
    assert out is not None and all(__import__("os").path.getsize(f) > 0 for f in out)
    import builtins
    real_import = builtins.__import__

    def no_mpl(name, *args, **kw):
        if name.startswith("matplotlib"):
            raise ImportError("no matplotlib")
        return real_import(name, *args, **kw)
    monkeypatch.setattr(builtins, "__import__", no_mpl)
    roc, pr = metrics.save_plots(y, p, str(tmp_path / "b"))
    assert roc.endswith(".svg") and "<polyline" in open(roc).read() and "AP =" in open(pr).read()


def test_binned_inference_equals_threshold_inference_on_new_rows():
    """Bins are cut at the trees' split thresholds: binned (folded-table / fp8-forest) inference
    on rows the model never saw equals the threshold walk — exactly for f64 tables, to the fp8
    two-term quantisation for the MFMA forest's operands."""
    from hfens.io.synth import make_hf_cohort
    from hfens.models.forest_infer import Fp8Forest, ensemble_raw_binned, stump_bin_tables
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.models.hist_gbdt import fit_gbdt_batch
    X, y, _ = make_hf_cohort(1500, 12, seed=71, nan_frac=0.0)
    Xn, _, _ = make_hf_cohort(700, 12, seed=72, nan_frac=0.0)
    X, y, Xn = torch.as_tensor(X), torch.as_tensor(y), torch.as_tensor(Xn)
    ms = [GradientBoostingClassifier(n_estimators=50, max_depth=1, random_state=s) for s in (1, 2)]
    fit_gbdt_batch(ms, X, y)
    bins = ms[0]._bin_mapper.transform(Xn)
    T, init = stump_bin_tables(ms)
    raw = ensemble_raw_binned(T, init, bins)
    for b, m in enumerate(ms):
        assert torch.allclose(raw[b], m.decision_function(Xn), atol=1e-9)
    m3 = [GradientBoostingClassifier(n_estimators=30, max_depth=3, random_state=3)]
    fit_gbdt_batch(m3, X, y)
    r8 = Fp8Forest(m3).reference_raw(m3[0]._bin_mapper.transform(Xn))
    assert float((r8[0] - m3[0].decision_function(Xn)).abs().max()) < 5e-3


def test_batched_bin_fit_matches_per_feature():
    """K7: the one-sort batched bin fit (device path) equals the per-feature distinct/quantile fit."""
    from hfens.io.synth import make_hf_cohort
    from hfens.models import binning
    X, _, _ = make_hf_cohort(5000, 20, seed=81, nan_frac=0.0)
    X = torch.as_tensor(X)
    X[:, 0] = torch.round(X[:, 0] * 3)          # few distinct values (some negative: sorted path)
    X[:, 1] = torch.arange(5000) % 40 + 3.0      # small non-negative integers: bincount path
    X[:, 2] = torch.arange(5000) % 300.0         # integers beyond 255: sorted path
    X32 = X.to(torch.float32)
    for mb in (256, 16):
        a = binning._fit_bins_device(X32, mb)
        b = binning.fit_bins(X, mb)
        assert torch.equal(a.nbins.cpu(), b.nbins.cpu())
        assert torch.equal(a.lo_val.cpu(), b.lo_val.cpu())
        assert torch.equal(a.hi_val.cpu(), b.hi_val.cpu())
        assert torch.equal(a.edges.cpu(), b.edges.cpu())
    a = binning._fit_bins_device(X32, 256)
    assert int(a.nbins.max()) == 256 and int(a.nbins.min()) <= 8 and int(a.nbins[1]) == 40


def test_knn_transform_many_equals_single_transforms():
    """transform_many (one host read for several matrices on the device path) is transform applied
    to each matrix."""
    from hfens.io.synth import make_hf_cohort
    from hfens.models.imputer import KNNImputer
    Xa, _, _ = make_hf_cohort(400, 9, seed=5, nan_frac=0.05)
    Xb, _, _ = make_hf_cohort(150, 9, seed=6, nan_frac=0.05)
    imp = KNNImputer(n_neighbors=1).fit(torch.as_tensor(Xa))
    a, b = imp.transform_many([torch.as_tensor(Xa), torch.as_tensor(Xb)])
    assert torch.equal(a, imp.transform(torch.as_tensor(Xa)))
    assert torch.equal(b, imp.transform(torch.as_tensor(Xb)))
    assert not torch.isnan(a).any() and not torch.isnan(b).any()


def test_cooperative_solver_member_policies(monkeypatch):
    """Member counts of the cooperative LR (CU budget while a cooperative SMO runs) and the GBDT
    stage-graph unit count (3-stage units while every stage still all-reduces)."""
    from hfens.models import hist_gbdt, logreg_solver
    monkeypatch.setattr(logreg_solver, "MEMBERS", 0)
    assert logreg_solver.lr_members(1, 10000, 256) == 16          # meta-LR: 16 row slabs
    assert logreg_solver.lr_members(6, 10000, 256) == 16
    assert logreg_solver.lr_members(1, 700, 256) == 2              # ≥ 512 rows per member
    monkeypatch.setattr(logreg_solver, "BLOCK_BUDGET", [30])
    assert logreg_solver.lr_members(6, 10000, 256) == 5            # 30 CUs left beside the SMO
    monkeypatch.setattr(logreg_solver, "MEMBERS", 1)
    assert logreg_solver.lr_members(6, 10000, 256) == 1

    class St:
        T = 100
    monkeypatch.setattr(hist_gbdt, "STAGE_GRAPH", "auto")
    assert hist_gbdt._graph_units(St, None, None) == 0            # single process: eager loop
    monkeypatch.setattr(hist_gbdt, "STAGE_GRAPH", "1")
    assert hist_gbdt._graph_units(St, None, None) == 33           # t = 0 … 98 replayed, 99 … 101 eager
    assert hist_gbdt._graph_units(St, None, object()) == 0        # stamps requested: eager
    St.T = 5
    assert hist_gbdt._graph_units(St, None, None) == 0            # too short to pay for a capture


def test_bin_edges_round_toward_the_lower_value():
    """a split threshold t = (a + c)/2 in f64 that rounds UP to a float32 t32 must not
    put x == t32 in the left bin — the threshold walk (x <= t, f64, as sklearn) sends it right."""
    import numpy as np
    from hfens.models.binning import _threshold_edges
    rng = np.random.default_rng(5)
    hits = 0
    for _ in range(2000):
        a, c = np.sort(rng.normal(size=2).astype(np.float32))
        if a == c:
            continue
        lo = torch.tensor([a, c], dtype=torch.float64)
        e = _threshold_edges(lo, lo, lo.to(torch.float32))
        t = float(a) / 2.0 + float(c) / 2.0
        t32 = np.float32(t)
        hits += float(t32) > t
        for x in (t32, np.nextafter(t32, np.float32(-np.inf)), np.nextafter(t32, np.float32(np.inf)), a, c):
            left_bin = float(x) <= float(e[0])
            left_walk = float(x) <= t
            assert left_bin == left_walk, (a, c, x)
    assert hits > 100      # the rounding-up case was exercised


def test_train_cli_reads_mat_next_to_script_and_plots(tmp_path, monkeypatch, capsys):
    """Reference no-arg behaviour (T:33-39, 66-90): the .mat files are read from the directory of
    the script that was run, not the working directory, and the ROC/PR figures are always drawn."""
    from hfens.cli.train_ensemble_public import main
    from hfens.io.mat import save_data
    from hfens.io.synth import make_dev_select
    Xd, yd, Xs, ys, names = make_dev_select(300, 24, seed=3)
    script_dir = tmp_path / "scriptdir"
    script_dir.mkdir()
    save_data(str(script_dir / "develop_data.mat"), Xd, yd, names)
    save_data(str(script_dir / "model_select_data.mat"), Xs, ys, names)
    work = tmp_path / "work"
    work.mkdir()
    monkeypatch.chdir(work)
    assert main(["--device", "cpu", "--json", str(work / "r.json")], script_dir=str(script_dir)) == 0
    out = capsys.readouterr().out
    assert "number of features =  17" in out and "not found" not in out
    import json
    assert json.loads(open(work / "r.json").read().splitlines()[-1])["source"] == "mat"
    made = sorted(p.name for p in work.iterdir())
    assert any(n.startswith("hf") and n.endswith((".png", ".svg")) for n in made), made

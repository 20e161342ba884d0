"""Checkpoint codec + CPU-exact inference goldens."""
import hashlib

import numpy as np
import pytest
import torch

from hfens.io import skpickle as sp
from hfens.io.checkpoint import checkpoint_graph, load_checkpoint, save_checkpoint
from hfens.cli.predict_hf import PATIENT_PARAMS, format_probability, predict_patient

MD5 = "b91deda0cf2c2b681ed39b2d472fe96f"
X0 = torch.tensor([[float(v) for v in PATIENT_PARAMS.values()]], dtype=torch.float64)


def _bytes(p):
    return open(p, "rb").read()


def test_fixture_is_the_shipped_checkpoint(ckpt_path):
    assert hashlib.md5(_bytes(ckpt_path)).hexdigest() == MD5


def test_ast_roundtrip_byte_exact(ckpt_path):
    b = _bytes(ckpt_path)
    assert sp.emit(sp.parse(b)) == b


def test_native_writer_byte_exact(ckpt_path, tmp_path):
    clf = load_checkpoint(ckpt_path)
    out = save_checkpoint(clf, str(tmp_path / "re.pkl"))
    assert len(out) == 132976
    assert out == _bytes(ckpt_path)


def test_parser_is_inert():
    # a pickle that would call os.system if executed; we must only build records
    evil = b"\x80\x03cos\nsystem\nq\x00X\x04\x00\x00\x00trueq\x01\x85q\x02Rq\x03."
    node = sp.parse(evil)
    assert isinstance(node, sp.Call) and node.func.module == "os"
    assert sp.emit(node) == evil


def test_schema(ckpt_path):
    clf = load_checkpoint(ckpt_path)
    svc = clf.estimators_[0].steps[1][1]
    assert svc.support_vectors_.shape == (434, 17)
    assert svc._n_support.tolist() == [321, 113]
    assert abs(svc._gamma - 1 / 17) < 1e-15
    gbc = clf.estimators_[1]
    assert gbc.n_estimators_ == 100 and gbc.tree_feature_.shape == (100, 3)
    assert abs(float(gbc.train_score_[0]) - 0.971894) < 1e-6
    assert abs(float(gbc.train_score_[-1]) - 0.755298) < 1e-6
    lg = clf.estimators_[2]
    assert float(lg.intercept_[0]) == 0.0 and int(lg.n_iter_[0]) == 48
    meta = clf.final_estimator_
    np.testing.assert_allclose(meta.coef_[0].numpy(), [1.8372434, 0.41020655, 2.88042418], rtol=1e-7)


def test_default_patient_golden(ckpt_path):
    p = predict_patient(model_path=ckpt_path)
    assert abs(p - 0.2709003) < 1e-7
    assert "27.09 %" in format_probability(p)


def test_branch_goldens(ckpt_path):
    clf = load_checkpoint(ckpt_path)
    meta = clf.transform(X0)[0].numpy()
    np.testing.assert_allclose(meta, [0.08854113, 0.09889406, 0.27639458], atol=1e-8)
    svc_dec = clf.estimators_[0].decision_function(X0)
    assert abs(float(svc_dec[0]) + 0.90725945) < 1e-7
    assert abs(float(clf.estimators_[1].decision_function(X0)[0]) + 2.2095736) < 1e-6


def test_svc_parity_with_installed_libsvm(ckpt_path):
    """sklearn 1.7.2's libsvm on the checkpoint's SVC parameters (trees are not
    loadable there; the SVC is): predict_proba must agree on random inputs."""
    svm = pytest.importorskip("sklearn.svm")
    clf = load_checkpoint(ckpt_path)
    pipe = clf.estimators_[0]
    scaler, m = pipe.steps[0][1], pipe.steps[1][1]
    sk = svm.SVC(C=1.0, kernel="rbf", gamma="scale", probability=True, class_weight="balanced")
    rng = np.random.default_rng(0)
    Xfit = rng.normal(size=(20, 17))
    yfit = np.r_[np.zeros(10), np.ones(10)]
    sk.fit(Xfit, yfit)
    sk.support_ = m.support_.numpy().astype(np.int32)
    sk.support_vectors_ = m.support_vectors_.numpy()
    sk._n_support = m._n_support.numpy().astype(np.int32)
    sk._dual_coef_ = m._dual_coef_.numpy()
    sk.dual_coef_ = m.dual_coef_.numpy()
    sk._intercept_ = m._intercept_.numpy()
    sk.intercept_ = m.intercept_.numpy()
    sk._probA = m._probA.numpy()
    sk._probB = m._probB.numpy()
    sk._gamma = m._gamma
    sk.shape_fit_ = m.shape_fit_
    sk.class_weight_ = m.class_weight_.numpy()
    X = np.vstack([X0.numpy(), rng.integers(0, 2, size=(50, 17)).astype(float)])
    X[:, 13] = rng.normal(18, 4, size=51)
    X[:, 16] = rng.normal(63, 5, size=51)
    Z = scaler.transform(torch.as_tensor(X)).numpy()
    ours = m.predict_proba(torch.as_tensor(Z))[:, 1].numpy()
    theirs = sk.predict_proba(Z)[:, 1]
    np.testing.assert_allclose(ours, theirs, atol=2e-8)


def _schema(v, path="root", out=None):
    """(path, class / dtype) signature of a value graph: state-dict key ORDER, estimator classes,
    array dtypes and ranks (shapes vary with the data)."""
    out = [] if out is None else out
    if isinstance(v, sp.SkObject):
        out.append((path, "obj", v.cls))
        if isinstance(v.state, dict):
            out.append((path, "keys", tuple(v.state)))
            for k, x in v.state.items():
                if k in ("estimators_",) and isinstance(x, np.ndarray) and x.dtype == object:
                    _schema(x.flat[0], f"{path}.{k}[0]", out)   # trees: one representative
                else:
                    _schema(x, f"{path}.{k}", out)
        if v.items:
            for k, x in v.items.items():
                _schema(x, f"{path}[{k}]", out)
    elif isinstance(v, np.ndarray):
        out.append((path, "arr", v.dtype.str if v.dtype != object else "O", v.ndim,
                    v.dtype.names or ()))
    elif isinstance(v, (list, tuple)):
        for i, x in enumerate(v):
            _schema(x, f"{path}[{i}]", out)
    elif isinstance(v, dict):
        out.append((path, "dict", tuple(v)))
        for k, x in v.items():
            _schema(x, f"{path}.{k}", out)
    elif isinstance(v, sp.NpRandomState):
        out.append((path, "rng", v.key.dtype.str, v.key.shape))
    else:
        out.append((path, "val", type(v).__name__))
    return out


@pytest.mark.parametrize("depth", [1, 3])
def test_trained_checkpoint_roundtrip(depth, tmp_path, ckpt_path):
    """develop-style fit → save_checkpoint → load_checkpoint gives identical f64
    predict_proba; depth > 1 trees are written in sklearn's compact depth-first node order; the
    fresh file's schema (classes, key order, dtypes) equals the shipped 0.23.2 checkpoint's."""
    from hfens.config import EnsembleConfig, build_estimators
    from hfens.io.synth import make_hf_cohort
    X, y, _ = make_hf_cohort(400, 17, seed=31, nan_frac=0.0)
    X, y = torch.as_tensor(X), torch.as_tensor(y)
    clf = build_estimators(EnsembleConfig(gbc_depth=depth))
    clf.fit(X, y)
    path = str(tmp_path / "fresh.pkl")
    save_checkpoint(clf, path)
    back = load_checkpoint(path)
    Xt, _, _ = make_hf_cohort(300, 17, seed=32, nan_frac=0.0)
    Xt = torch.as_tensor(Xt)
    assert torch.equal(back.predict_proba(Xt), clf.predict_proba(Xt))
    fresh = sp.to_py(sp.parse(_bytes(path)))
    shipped = sp.to_py(sp.parse(_bytes(ckpt_path)))
    assert _schema(fresh) == _schema(shipped)
    # compact depth-first trees: every node reachable, children after their parent, left first
    for est in fresh.state["estimators_"][1].state["estimators_"][:, 0]:
        nodes = est.state["tree_"].state["nodes"]
        assert est.state["tree_"].state["node_count"] == len(nodes)
        for i, nd in enumerate(nodes):
            if nd["left_child"] >= 0:
                assert nd["left_child"] == i + 1 and nd["right_child"] > nd["left_child"]
            else:
                assert nd["feature"] == -2 and nd["right_child"] == -1
    # and a re-save of the loaded model reproduces the fresh file byte for byte
    assert save_checkpoint(back, str(tmp_path / "again.pkl")) == _bytes(path)

"""Host-side bookkeeping of the working-set SMO (models/smo.py) that needs no GPU."""
import numpy as np
import pytest


@pytest.mark.parametrize("l,npos", [(10000, 2300), (8000, 1841), (6400, 3200), (4096, 5), (4500, 4000)])
def test_cascade_parts_partition_the_problem(l, npos):
    """smo.cascade_parts: disjoint parts covering every point once, each class-stratified (its
    positives first, as a problem's layout requires) — so the concatenated part solutions are a
    feasible point of the full problem (same C, Σ yα = 0 per part)."""
    from hfens.models import smo
    p = smo._Prob(0, -1, np.arange(l), npos, 1.0, 1.0, 0.1)
    parts = smo.cascade_parts(p)
    P = smo.cascade_split(l, npos)
    assert len(parts) == P
    if P == 0:
        return
    allpos = np.concatenate(parts)
    assert np.array_equal(np.sort(allpos), np.arange(l))
    for pos in parts:
        cp = int((pos < npos).sum())
        assert np.all(pos[:cp] < npos) and np.all(pos[cp:] >= npos)
        assert abs(cp - npos / P) <= 1 and abs((pos.shape[0] - cp) - (l - npos) / P) <= 1


@pytest.mark.parametrize("n,p1,seed", [(10000, 0.2, 2020), (713, 0.198, 7), (37, 0.05, 3), (12, 0.1, 1), (9, 0.0, 5)])
def test_native_expand_matches_numpy(n, p1, seed):
    """ops/csrc/host.hip svc_expand_host (one native call per fit, the stacking plan's hot loop)
    equals the numpy expansion array for array: grouped positions, Platt folds' training rows in
    permutation order (class 1 first), held-out positions and rows, class counts, constant folds."""
    from hfens import ops
    from hfens.models import smo
    from hfens.models.svc import SVC
    if not ops.has_ext():
        pytest.skip("extension not built")
    rng = np.random.default_rng(seed)
    y = (rng.random(n) < p1).astype(np.float64)
    for prob in (True, False):
        svc = SVC(class_weight="balanced", probability=prob, random_state=seed)
        cw = np.array([0.7, 2.1])
        a, ma = smo._expand_native(0, y, 0.25, cw, svc)
        b, mb = smo._expand_py(0, y, 0.25, cw, svc)
        assert len(a) == len(b)
        assert ma["n0"] == mb["n0"] and ma["l"] == mb["l"] and np.array_equal(ma["grouped"], mb["grouped"])
        for p, q in zip(a, b):
            assert (p.fold, p.npos, p.Cp, p.Cn, p.const) == (q.fold, q.npos, q.Cp, q.Cn, q.const)
            for f in ("rows", "held", "held_rows"):
                u, v = getattr(p, f), getattr(q, f)
                assert (u is None) == (v is None)
                if u is not None:
                    assert np.array_equal(u, v), f


@pytest.mark.parametrize("n,p1,seed", [(10000, 0.2, 1), (713, 0.198, 2), (23, 0.5, 3), (11, 0.3, 4)])
def test_stratified_binary_fast_path_matches_generic(n, p1, seed):
    """model_selection._stratified_binary (the stacking plan's folds in a few vector ops) gives
    StratifiedKFold's assignment exactly as the generic np.unique path does, whichever class
    appears first."""
    from hfens.models import model_selection as ms
    rng = np.random.default_rng(seed)
    for first in (0.0, 1.0):
        y = (rng.random(n) < p1).astype(np.float64)
        y[0] = first
        if len(np.unique(y)) < 2:
            continue
        assert np.array_equal(ms._stratified_binary(y, 5), ms._stratified_generic(y, 5))
    assert ms._stratified_binary(np.array([0.0, 1.0, 2.0, 1.0, 0.0, 2.0]), 2) is None


@pytest.mark.parametrize("n,p1,seed", [(10000, 0.2, 2020), (5003, 0.198, 7), (4300, 0.3, 3), (713, 0.2, 4)])
def test_native_stacking_plan_matches_python(n, p1, seed):
    """stack_trainer.plan_stacking_start (ONE GIL-free native call on a helper thread: StratifiedKFold
    test folds of two-class labels + every fit's libsvm expansion) gives plan_stacking's plan array for
    array, whichever class is seen first (below the working-set solver's size the stored-Gram solver's
    column maps keep the Python plan: None)."""
    from hfens import ops
    from hfens.config import EnsembleConfig, build_estimators
    from hfens.models import stack_trainer
    if not ops.has_ext():
        pytest.skip("extension not built")
    clf = build_estimators(EnsembleConfig())
    rng = np.random.default_rng(seed)
    for first in (0.0, 1.0):
        y = (rng.random(n) < p1).astype(np.float64)
        y[0] = first
        join = stack_trainer.plan_stacking_start(clf, y)
        from hfens.models import smo
        if n < smo.WS_MIN_POINTS:
            assert join is None
            continue
        assert join is not None
        a, b = join(), stack_trainer.plan_stacking(clf, y)
        assert np.array_equal(a["folds_np"], b["folds_np"])
        assert all(np.array_equal(u, v) for u, v in zip(a["rows_host"], b["rows_host"]))
        assert a["svc_pre"].keys() == b["svc_pre"].keys()
        for k in a["svc_pre"]:
            for (ya, pa, ma), (yb, pb, mb) in zip(a["svc_pre"][k], b["svc_pre"][k]):
                assert np.array_equal(ya, yb) and ma["n0"] == mb["n0"] and np.array_equal(ma["grouped"], mb["grouped"])
                assert (ma["C0"], ma["C1"]) == (mb["C0"], mb["C1"])
                for p, q in zip(pa, pb):
                    assert (p.fit, p.fold, p.npos, p.Cp, p.Cn, p.const) == (q.fit, q.fold, q.npos, q.Cp, q.Cn, q.const)
                    for f in ("rows", "held", "held_rows"):
                        u, v = getattr(p, f), getattr(q, f)
                        assert (u is None) == (v is None) and (u is None or np.array_equal(u, v))

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


def test_gather_rows_single_gather_matches_per_fit():
    """smo._gather_rows: when every fit's matrix is a row block of one matrix (the batched scaler's
    output) the one-gather path returns exactly the per-fit gathers' concatenation."""
    import torch
    from hfens.models import smo

    class P:
        def __init__(self, fit, rows):
            self.fit, self.rows = fit, rows
    rng = np.random.default_rng(0)
    Z = torch.randn(150, 4, dtype=torch.float64)
    blocks = [Z[0:50], Z[50:100], Z[100:150]]
    probs = [P(f, rng.integers(0, 50, size=int(rng.integers(5, 30))).astype(np.int64)) for f in (0, 0, 1, 2, 2, 2)]
    one = smo._gather_rows(blocks, probs, "rows", "cpu")
    per_fit = smo._gather_rows([b.clone() for b in blocks], probs, "rows", "cpu")
    assert one.dtype == torch.float32 and torch.equal(one, per_fit)


def test_cascade_tables_match_the_per_problem_split():
    """smo._cascade_tables (vectorised) equals the per-problem loop over cascade_split: the parts
    table rows (start, length, parent offset, P, j, parent npos, part npos) and every part's record."""
    from hfens.models import smo
    rng = np.random.default_rng(5)
    sizes = [10000, 8000, 8000, 6400, 6400, 4096, 4095, 4500, 5000, 3000, 12345, 5201]
    live, aoffs = [], [0]
    for k, l in enumerate(sizes):
        npos = int(rng.integers(1, l)) if k != 7 else 2       # (k = 7: too few positives to split)
        live.append(smo._Prob(k % 6, k % 5 - 1, np.arange(l), npos, 1.0 + 0.1 * k, 0.7 + 0.05 * k, 0.05 + 0.01 * k))
        aoffs.append(aoffs[-1] + l)
    tab, start = [], 0
    ref = []
    for k, p in enumerate(live):
        P = smo.cascade_split(p.l, p.npos)
        for j in range(P):
            cp, cn = (p.npos - j + P - 1) // P, (p.l - p.npos - j + P - 1) // P
            tab.append((start, cp + cn, aoffs[k], P, j, p.npos, cp))
            ref.append((p.fit, p.fold, cp + cn, cp, p.Cp, p.Cn, p.gamma))
            start += cp + cn
    got_tab, parts = smo._cascade_tables(live, aoffs)
    assert got_tab.dtype == np.int64 and np.array_equal(got_tab, np.asarray(tab, dtype=np.int64))
    assert len(parts) == len(ref) and parts.max_l == max(r[2] for r in ref)
    for k, r in enumerate(ref):
        q = parts[k]
        assert (q.fit, q.fold, q.l, q.npos, q.Cp, q.Cn, q.gamma) == r
    assert smo._cascade_tables([live[7]], [0, live[7].l]) is None


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

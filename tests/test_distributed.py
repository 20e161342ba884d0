"""Data-parallel paths on the CPU with gloo (world_size 2): sharded training must
reproduce the single-process fit (GBDT bit-identically thanks to fixed-point
histograms)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _plain(x):
    """Tensors -> numpy before crossing the queue: a torch tensor is sent as a shared-memory
    handle that dies with the worker, so the parent could read it after rank 0 exited."""
    if isinstance(x, torch.Tensor):
        return _T(x.detach().cpu().numpy())
    if isinstance(x, (tuple, list)):
        return type(x)(_plain(v) for v in x)
    if isinstance(x, dict):
        return {k: _plain(v) for k, v in x.items()}
    return x


class _T:
    def __init__(self, a):
        self.a = a


def _unplain(x):
    if isinstance(x, _T):
        return torch.from_numpy(x.a)
    if isinstance(x, (tuple, list)):
        return type(x)(_unplain(v) for v in x)
    if isinstance(x, dict):
        return {k: _unplain(v) for k, v in x.items()}
    return x


def _worker(rank, world, port, fn_name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = globals()[fn_name](rank, world, dist.group.WORLD)
        if rank == 0:
            q.put(_plain(out))
    finally:
        dist.destroy_process_group()


def _worker_nccl(rank, world, port, fn_name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), HFENS_DIST_BACKEND="nccl")
    from hfens.parallel import dist as pdist
    group, r, w = pdist.init_from_env()
    try:
        out = globals()[fn_name](r, w, group)
        if rank == 0:
            q.put(_plain(out))
    finally:
        pdist.shutdown()


def _nccl_sum(rank, world, group):
    from hfens.parallel import dist as pdist
    t = torch.full((2,), float(rank + 1), device=pdist.rank_device())
    pdist.all_reduce_sum_(t, group)
    return t.cpu().tolist()


def _run_nccl(fn_name, world):
    return _run(fn_name, world, target=_worker_nccl)


def _run(fn_name, world=2, target=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target or _worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue as _q
    out = None
    while out is None:
        try:
            out = q.get(timeout=2)
        except _q.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                for p in procs:
                    p.kill()
                raise RuntimeError(f"worker failed: {[p.exitcode for p in procs]}")
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return _unplain(out)


def _data(n=1200, F=20, seed=3):
    from hfens.io.synth import make_hf_cohort
    X, y, names = make_hf_cohort(n, F, seed=seed, nan_frac=0.0)
    return torch.as_tensor(X), torch.as_tensor(y), names


def _gbdt(rank, world, group):
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.models.hist_gbdt import fit_gbdt_batch
    from hfens.parallel.dist import shard_rows
    X, y, _ = _data()
    masks = torch.ones(2, X.shape[0], dtype=torch.bool)
    masks[0, ::4] = False
    ms = [GradientBoostingClassifier(n_estimators=15, max_depth=2) for _ in range(2)]
    fit_gbdt_batch(ms, shard_rows(X, rank, world), shard_rows(y, rank, world),
                   shard_rows(masks.t(), rank, world).t().contiguous(), group=group)
    return [(m.tree_feature_.clone(), m.tree_threshold_.clone(), m.tree_value_.clone(), m.train_score_.clone(),
             m.tree_impurity_.clone()) for m in ms]


def _gbdt_sub(rank, world, group):
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.models.hist_gbdt import fit_gbdt_batch
    from hfens.parallel.dist import shard_rows
    X, y, _ = _data()
    ms = [GradientBoostingClassifier(n_estimators=12, max_depth=2, subsample=0.6, random_state=s) for s in (1, 2)]
    fit_gbdt_batch(ms, shard_rows(X, rank, world), shard_rows(y, rank, world), group=group)
    return [(m.tree_feature_.clone(), m.tree_threshold_.clone(), m.tree_value_.clone(), m.train_score_.clone())
            for m in ms]


def _logreg(rank, world, group):
    from hfens.models.linear import LogisticRegression
    from hfens.models.logreg_solver import fit_logreg_batch
    from hfens.parallel.dist import shard_rows
    X, y, _ = _data()
    m = LogisticRegression(penalty="l1", solver="liblinear", class_weight="balanced")
    fit_logreg_batch([m], shard_rows(X, rank, world), shard_rows(y, rank, world), group=group)
    return m.coef_.clone(), m.intercept_.clone()


def _lasso(rank, world, group):
    from hfens.models.lasso import LassoCV, SelectFromModel
    from hfens.parallel.dist import shard_rows
    X, y, _ = _data()
    s = SelectFromModel(LassoCV(cv=10), threshold=-np.inf, max_features=8)
    s.fit(shard_rows(X, rank, world), shard_rows(y, rank, world), group=group)
    return s.estimator_.alpha_, s.estimator_.coef_.clone(), s.get_support().copy()


def _develop(rank, world, group, policy="dp"):
    from hfens import pipeline
    from hfens.io.synth import make_dev_select
    from hfens.parallel.dist import shard_rows
    from hfens.pipeline import develop
    pipeline.DP_POLICY = policy
    Xd, yd, Xs, ys, names = make_dev_select(600, 30, seed=5)
    r = develop(shard_rows(Xd, rank, world), shard_rows(yd, rank, world), shard_rows(Xs, rank, world),
                shard_rows(ys, rank, world), names, device="cpu", group=group)
    from hfens.parallel.dist import all_gather_rows
    p = all_gather_rows(r.proba_sel.double()[:, None], group)[:, 0]
    return r.selected.copy(), r.scores, p


def _develop_task(rank, world, group):
    return _develop(rank, world, group, policy="task")


def _svc_task(rank, world, group):
    """Task-parallel SMO: problems spread over the ranks by assign_problems, solutions all-reduced."""
    from hfens.models.smo import fit_svc_batch
    from hfens.models.svc import SVC
    X, y, _ = _data(300, 8, seed=9)
    Z = (X - X.mean(0)) / X.std(0, unbiased=False)
    Zs, ys = [Z[:240], Z], [y[:240], y]
    svcs = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in Zs]
    fit_svc_batch(svcs, Zs, ys, group=group)
    return [(s._dual_coef_.clone(), float(s._intercept_[0]), s._probA.item(), s._probB.item()) for s in svcs]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gbdt_dp_bit_identical(world):
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.models.hist_gbdt import fit_gbdt_batch
    got = _run("_gbdt", world)
    X, y, _ = _data()
    masks = torch.ones(2, X.shape[0], dtype=torch.bool)
    masks[0, ::4] = False
    ms = [GradientBoostingClassifier(n_estimators=15, max_depth=2) for _ in range(2)]
    fit_gbdt_batch(ms, X, y, masks)
    for (f, t, v, ts, imp), m in zip(got, ms):
        assert torch.equal(f, m.tree_feature_)
        assert torch.equal(t, m.tree_threshold_)
        assert torch.equal(v, m.tree_value_)
        assert torch.equal(ts, m.train_score_)
        assert torch.equal(imp, m.tree_impurity_)   # leaf impurities are global sums too


def test_gbdt_subsample_dp_bit_identical():
    """Counter-based bagging keyed by the global row index: the same stochastic GB for any sharding."""
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.models.hist_gbdt import fit_gbdt_batch
    got = _run("_gbdt_sub")
    X, y, _ = _data()
    ms = [GradientBoostingClassifier(n_estimators=12, max_depth=2, subsample=0.6, random_state=s) for s in (1, 2)]
    fit_gbdt_batch(ms, X, y)
    assert not torch.equal(ms[0].tree_value_, ms[1].tree_value_)   # seeds give different bags
    for (f, t, v, ts), m in zip(got, ms):
        assert torch.equal(f, m.tree_feature_)
        assert torch.equal(t, m.tree_threshold_)
        assert torch.equal(v, m.tree_value_)
        assert torch.equal(ts, m.train_score_)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_logreg_dp(world):
    from hfens.models.linear import LogisticRegression
    from hfens.models.logreg_solver import fit_logreg_batch
    coef, ic = _run("_logreg", world)
    X, y, _ = _data()
    m = LogisticRegression(penalty="l1", solver="liblinear", class_weight="balanced")
    fit_logreg_batch([m], X, y)
    assert torch.allclose(coef, m.coef_, atol=1e-8)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_lasso_dp(world):
    from hfens.models.lasso import LassoCV, SelectFromModel
    alpha, coef, sup = _run("_lasso", world)
    X, y, _ = _data()
    s = SelectFromModel(LassoCV(cv=10), threshold=-np.inf, max_features=8).fit(X, y)
    assert abs(alpha - s.estimator_.alpha_) < 1e-15
    assert np.array_equal(sup, s.get_support())
    assert torch.allclose(coef, s.estimator_.coef_, atol=1e-10)


def test_assign_problems_lpt():
    """The largest SMO problem (the critical path) owns rank 0 alone; the rest are spread
    longest-first over ranks 1 … W−1; one rank keeps everything."""
    from hfens.models.smo import assign_problems
    sizes = [10, 8, 8, 8, 8, 8, 6, 6]
    own = assign_problems(sizes, 4)
    assert own[0] == 0 and own.count(0) == 1 and sorted(set(own)) == [0, 1, 2, 3]
    loads = [sum(s for s, o in zip(sizes, own) if o == r) for r in range(1, 4)]
    assert max(loads) - min(loads) <= 6
    assert assign_problems(sizes, 1) == [0] * len(sizes)
    assert assign_problems(sizes, 2) == [0] + [1] * 7
    assert assign_problems([5], 3) == [0]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_svc_task_parallel_matches_single(world):
    from hfens.models.smo import fit_svc_batch
    from hfens.models.svc import SVC
    got = _run("_svc_task", world)
    X, y, _ = _data(300, 8, seed=9)
    Z = (X - X.mean(0)) / X.std(0, unbiased=False)
    svcs = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in range(2)]
    fit_svc_batch(svcs, [Z[:240], Z], [y[:240], y])
    for (coef, ic, a, b), s in zip(got, svcs):
        assert torch.equal(coef, s._dual_coef_)
        assert ic == float(s._intercept_[0]) and a == s._probA.item() and b == s._probB.item()


@pytest.mark.parametrize("world", [2, 8])
def test_develop_task_matches_single(world):
    """'task' policy (rows gathered once, the SMO problems spread over ranks): every rank fits on
    the full rows, so the model equals the single-process one bit for bit.  The held-out rows are
    scored per shard: ≤ 256 rows go through the native f64 host predictor, more through the
    per-model torch path — the same f64 formula, equal to 1e-12 (at world 8: 75-row shards)."""
    from hfens.io.synth import make_dev_select
    from hfens.pipeline import develop
    sel, scores, p = _run("_develop_task", world)
    Xd, yd, Xs, ys, names = make_dev_select(600, 30, seed=5)
    r = develop(Xd, yd, Xs, ys, names, device="cpu")
    assert np.array_equal(sel, r.selected)
    assert float((p - r.proba_sel.double()).abs().max()) <= 1e-12
    if world == 2:   # 300-row shards: the same predict path as the single process
        assert torch.equal(p, r.proba_sel.double())
    assert abs(scores["auroc"] - r.scores["auroc"]) <= 1e-12


@pytest.mark.parametrize("world", [2, 4, 8])
def test_develop_dp_matches_single(world):
    """'dp' policy (rows stay sharded): the integer reductions (GBDT histograms, KNN donors,
    AUROC) are exact; the f64 sums (LassoCV Grams, scaler moments, LR Newton moments) are summed
    in a rank-count-dependent order, which moves them by a few ulp.  Pinned here: the same
    selected features and held-out probabilities within 1e-12 of the single-process fit
    (measured: ≤ 4.4e-16) at 2, 4 and 8 ranks (parallel/dist.py states the bound)."""
    from hfens.io.synth import make_dev_select
    from hfens.pipeline import develop
    sel, scores, p = _run("_develop", world)
    Xd, yd, Xs, ys, names = make_dev_select(600, 30, seed=5)
    r = develop(Xd, yd, Xs, ys, names, device="cpu")
    assert np.array_equal(sel, r.selected)
    assert float((p - r.proba_sel.double()).abs().max()) <= 1e-12
    assert abs(scores["auroc"] - r.scores["auroc"]) <= _tie_slack(r.proba_sel.double(), ys)


def _tie_slack(p, y, tol=1e-12):
    """AUROC is a step function of the score order: probabilities equal to 1e-12 can still swap
    a cross-class pair whose scores TIE to within that tolerance (rows with equal features scored
    in different shard batches).  Each such pair moves the AUROC by at most 1/(n_pos n_neg)."""
    p = torch.as_tensor(p, dtype=torch.float64)
    y = torch.as_tensor(np.asarray(y).ravel() > 0)
    pos, neg = p[y], p[~y]
    near = int(((pos[:, None] - neg[None, :]).abs() <= 2 * tol).sum())
    return 1e-12 + near / (len(pos) * len(neg))


def _stack_dp(rank, world, group, lowrank=False):
    from hfens.models import smo
    from hfens.models.stacking import StackingClassifier
    from hfens.config import EnsembleConfig, build_estimators
    from hfens.parallel.dist import shard_rows
    if lowrank:
        smo.SOLVER = "lowrank"
    X, y, _ = _data(480, 8, seed=13)
    clf = build_estimators(EnsembleConfig())
    clf.fit(shard_rows(X, rank, world), shard_rows(y, rank, world), group=group)
    if lowrank:
        from hfens.models import svc_lowrank
        assert svc_lowrank.LAST_INFO.get("row_sharded") is True
    sc = clf.estimators_[0].steps[0][1]
    svc = clf.estimators_[0].steps[-1][1]
    return (sc.mean_.clone(), sc.scale_.clone(), svc._dual_coef_.clone(), float(svc._intercept_[0]),
            svc.support_.clone(), clf.final_estimator_.coef_.clone())


def _stack_dp_lowrank(rank, world, group):
    return _stack_dp(rank, world, group, lowrank=True)


def _svc_broadcast(rank, world, group):
    """broadcast_svc_fits alone: every rank fits the same 6 SVCs, then each fit is replaced by its
    owner's through the packed broadcast; returns every fit's state and the collective count."""
    from hfens.models.smo import fit_svc_batch
    from hfens.models.svc import SVC
    from hfens.parallel import stack
    X, y, _ = _data(300, 8, seed=21)
    Z = (X - X.mean(0)) / X.std(0, unbiased=False)
    Zs = [Z[30 * k:] for k in range(6)]
    ys = [y[30 * k:] for k in range(6)]
    svcs = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in Zs]
    fit_svc_batch(svcs, Zs, ys)
    # scramble the non-owned fits so that only the broadcast can restore them
    for f, s in enumerate(svcs):
        if f % world != rank:
            s._dual_coef_ = s._dual_coef_ * 0.0 + 7.0
            s._gamma = -1.0
    stack.broadcast_svc_fits(svcs, Zs, group)
    return ([(s.support_.clone(), s.support_vectors_.clone(), s._dual_coef_.clone(), float(s._intercept_[0]),
              float(s._probA[0]), float(s._probB[0]), s._gamma, s.shape_fit_, s._n_support.clone())
             for s in svcs], stack.COLLECTIVES["broadcast_svc_fits"])


@pytest.mark.parametrize("world", [2, 4])
def test_broadcast_svc_fits_packed(world):
    """the task-parallel SVC fits travel in TWO collectives for all six fits
    (shape table + one packed f64 SUM), bit-exact: every rank ends with the owner's arrays."""
    got, ncoll = _run("_svc_broadcast", world)
    from hfens.models.smo import fit_svc_batch
    from hfens.models.svc import SVC
    X, y, _ = _data(300, 8, seed=21)
    Z = (X - X.mean(0)) / X.std(0, unbiased=False)
    Zs = [Z[30 * k:] for k in range(6)]
    ys = [y[30 * k:] for k in range(6)]
    ref = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in Zs]
    fit_svc_batch(ref, Zs, ys)
    assert ncoll == 2
    for g, s in zip(got, ref):
        sup, sv, coef, ic, pa, pb, gam, shp, ns = g
        assert torch.equal(sup.to(torch.int32), s.support_) and torch.equal(sv, s.support_vectors_)
        assert torch.equal(coef, s._dual_coef_) and ic == float(s._intercept_[0])
        assert pa == float(s._probA[0]) and pb == float(s._probB[0]) and gam == s._gamma
        assert tuple(shp) == tuple(s.shape_fit_) and torch.equal(ns.to(torch.int32), s._n_support.to(torch.int32))


def _stack_single(lowrank=False):
    from hfens.models import smo
    from hfens.config import EnsembleConfig, build_estimators
    old = smo.SOLVER
    smo.SOLVER = "lowrank" if lowrank else old
    try:
        X, y, _ = _data(480, 8, seed=13)
        clf = build_estimators(EnsembleConfig())
        clf.fit(X, y)
    finally:
        smo.SOLVER = old
    sc = clf.estimators_[0].steps[0][1]
    svc = clf.estimators_[0].steps[-1][1]
    return sc, svc, clf


@pytest.mark.parametrize("world", [2, 4, 8])
def test_stack_dp_scaler_and_svc_match_single(world):
    """the DP stack's StandardScaler moments are reduced over ALL ranks, so the
    scaled rows, the SVC solution and the meta-learner equal the single-process fit."""
    mean, scale, coef, ic, sup, meta = _run("_stack_dp", world)
    sc, svc, clf = _stack_single()
    assert torch.allclose(mean, sc.mean_, rtol=0, atol=1e-12)
    assert torch.allclose(scale, sc.scale_, rtol=0, atol=1e-12)
    assert torch.equal(sup, svc.support_)
    assert torch.allclose(coef, svc._dual_coef_, atol=1e-9)
    assert abs(ic - float(svc._intercept_[0])) < 1e-9
    assert torch.allclose(meta, clf.final_estimator_.coef_, atol=1e-6)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_stack_dp_lowrank_svc_matches_single(world):
    """The large-problem SVC path (Nyström + IPM) under DP, row-sharded:
    every rank holds only its rows of Φ and every interior-point solve all-reduces its row sums;
    the fit equals the single-process low-rank fit to 1e-8 (only the rank count's summation order
    of those sums differs).  At world 8 the 480-row cohort gives 60-row shards, so some ranks own
    no landmark and some Platt folds hold no row of a rank (empty local problems)."""
    mean, scale, coef, ic, sup, meta = _run("_stack_dp_lowrank", world)
    sc, svc, clf = _stack_single(lowrank=True)
    assert torch.equal(sup, svc.support_)
    assert torch.allclose(coef, svc._dual_coef_, rtol=0, atol=1e-8)
    assert abs(ic - float(svc._intercept_[0])) < 1e-8
    assert torch.allclose(meta, clf.final_estimator_.coef_, rtol=0, atol=1e-8)


def test_nccl_all_reduce_two_gpus():
    """The RCCL (backend "nccl") branch of hfens.parallel.dist with ≥ 2 visible GPUs."""
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    got = _run_nccl("_nccl_sum", 2)
    assert got == [3.0, 3.0]


def _auc_sharded(rank, world, group):
    from hfens.parallel.dist import shard_rows
    from hfens.utils import metrics
    rng = np.random.default_rng(17)
    y = (rng.random(3001) < 0.3).astype(np.float64)
    s = np.round(rng.random(3001) * 0.6 + 0.3 * y, 3)          # heavy ties, some cross-class
    s[:40] = 0.5                                               # one big tie block
    out = []
    for bins in (1 << 16, 8):                                  # fine grid, and a grid of all-mixed buckets
        out.append(metrics.roc_auc_sharded(shard_rows(torch.as_tensor(y), rank, world),
                                           shard_rows(torch.as_tensor(s), rank, world), group, bins=bins))
    # every score tied: one bucket holds all rows (the sort path, no pairwise matrix) → exactly ½
    out.append(metrics.roc_auc_sharded(shard_rows(torch.as_tensor(y), rank, world),
                                       shard_rows(torch.full((3001,), 0.25, dtype=torch.float64), rank, world), group))
    return torch.tensor(out), torch.tensor([metrics.roc_auc(torch.as_tensor(y), torch.as_tensor(s))])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_roc_auc_sharded_is_exact(world):
    """R8: the bucket-count all-reduce AUROC equals the single-process (sklearn-equal) AUROC exactly
    (ties inside mixed buckets resolved from their gathered rows)."""
    got, want = _run("_auc_sharded", world)
    assert abs(float(got[0]) - float(want[0])) < 1e-15
    assert abs(float(got[1]) - float(want[0])) < 1e-15
    assert float(got[2]) == 0.5


def _bin_data():
    g = np.random.default_rng(11)
    n = 1003
    X = np.empty((n, 7), dtype=np.float64)
    X[:, 0] = g.normal(size=n) * 1e3                          # continuous, negatives
    X[:, 1] = g.integers(0, 2, n)                             # binary
    X[:, 2] = np.where(np.arange(n) < n // 2, g.integers(0, 200, n), g.integers(200, 400, n))  # ≤ 256 per shard, 400 total
    X[:, 3] = np.round(g.normal(size=n), 1)                   # heavy ties across shards
    X[:, 4] = np.where(g.random(n) < 0.5, 0.0, -0.0)          # ±0: one value
    X[:, 5] = np.sort(g.exponential(size=n))                  # sorted: each shard holds a value range
    X[:, 6] = g.integers(0, 100, n)                           # small integers: bincount path (> 16 values: quantiles at mb 16)
    return torch.as_tensor(X)


def _bins_dp(rank, world, group):
    from hfens.models.binning import fit_bins
    from hfens.parallel.dist import shard_rows
    X = _bin_data()
    out = []
    for mb in (256, 16):
        bm = fit_bins(shard_rows(X, rank, world), mb, group=group)
        out.append((bm.nbins.clone(), bm.lo_val.clone(), bm.hi_val.clone(), bm.edges.clone()))
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_fit_bins_dp_equals_single_process(world):
    """K7 under DP: order-statistic bisection over all-reduced counts gives the single-process bins
    (quantile and one-bin-per-value features, ties across shards, ±0, a 400-value union of two
    ≤ 256-value shards, value ranges split by shard)."""
    from hfens.models.binning import fit_bins
    got = _run("_bins_dp", world)
    X = _bin_data()
    for (nb, lo, hi, e), mb in zip(got, (256, 16)):
        bm = fit_bins(X, mb)
        assert torch.equal(nb, bm.nbins)
        assert torch.equal(lo, bm.lo_val)
        assert torch.equal(hi, bm.hi_val)
        assert torch.equal(e, bm.edges)


def _seed_ens(rank, world, group):
    """Every seed-group layout S (ranks per group) of 5 seeds: each rank trains its seeds (on its
    row shard of the group) and the trees of every seed are all-gathered as int64/f64 rows."""
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.parallel import ensemble
    X, y, _ = _data(1500, 12, 9)
    out = {}
    for S in [s for s in (1, 2, 4, 8) if world % s == 0]:
        ms = [GradientBoostingClassifier(n_estimators=8, max_depth=1, subsample=0.7, random_state=10 + k)
              for k in range(5)]
        mine = ensemble.fit_seed_ensemble(ms, X, y, rank, world, S, group)
        # one row per (seed, tree): [seed, feature, threshold, value0..2, train_score]; group
        # leaders contribute, everyone else sends nothing
        rows = []
        if rank % S == 0:
            for k in mine:
                m = ms[k]
                for t in range(8):
                    rows.append([k, float(m.tree_feature_[t, 0]), float(m.tree_threshold_[t, 0])]
                                + [float(v) for v in m.tree_value_[t].reshape(-1)[:3]] + [float(m.train_score_[t])])
        loc = torch.tensor(rows, dtype=torch.float64).reshape(-1, 7)
        from hfens.parallel.dist import all_gather_rows
        allr = all_gather_rows(loc, group)
        out[S] = allr[torch.argsort(allr[:, 0] * 100 + torch.arange(allr.shape[0]) % 8, stable=True)]
    return out


@pytest.mark.parametrize("world", [2, 4, 8])
def test_seed_parallel_bit_identical(world):
    """Seed / hybrid / row layouts of a 5-seed bagged ensemble (parallel/ensemble.py, BASELINE
    config 5): every seed's trees, leaf values and train scores equal the single-process batched
    fit bit for bit (S = 1: whole seeds per rank, no collective; S = world: rows sharded)."""
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.models.hist_gbdt import fit_gbdt_batch
    got = _run("_seed_ens", world)
    X, y, _ = _data(1500, 12, 9)
    ms = [GradientBoostingClassifier(n_estimators=8, max_depth=1, subsample=0.7, random_state=10 + k)
          for k in range(5)]
    fit_gbdt_batch(ms, X, y)
    want = torch.tensor([[k, float(m.tree_feature_[t, 0]), float(m.tree_threshold_[t, 0])]
                         + [float(v) for v in m.tree_value_[t].reshape(-1)[:3]] + [float(m.train_score_[t])]
                         for k, m in enumerate(ms) for t in range(8)], dtype=torch.float64)
    assert set(got) == {s for s in (1, 2, 4, 8) if world % s == 0}
    for S, rows in got.items():
        assert rows.shape == want.shape, (S, rows.shape)
        assert torch.equal(rows, want), S


def test_seed_layout_cost_model():
    from hfens.parallel import ensemble
    assert ensemble.seed_layout(8, 1, 1_000_000) == 8          # one seed: shard its rows
    assert ensemble.seed_layout(8, 5, 1_000_000, "seeds") == 1
    assert ensemble.seed_layout(8, 5, 1_000_000, "rows") == 8
    assert ensemble.seed_layout(8, 5, 1_000_000, "4") == 4
    S = ensemble.seed_layout(8, 5, 1_000_000)
    assert 8 % S == 0
    assert ensemble.my_seeds(0, 8, 5, 1) == [0] and ensemble.my_seeds(5, 8, 5, 1) == []
    assert ensemble.my_seeds(4, 8, 5, 4) == [1, 3] and ensemble.my_seeds(3, 8, 5, 4) == [0, 2, 4]
    with pytest.raises(ValueError):
        ensemble.seed_layout(8, 5, 1000, "3")


def _ipm_batched(rank, world, group):
    """Three row-sharded interior-point problems (different sizes): solved one after another
    (ipm_svc_dual, a collective per reduction of each) and in lock-step (_drive, one collective per
    reduction step for all of them)."""
    from hfens.models import svc_lowrank as sl
    g = torch.Generator().manual_seed(5)
    probs = []
    for l in (900, 700, 500):
        Phi = torch.randn(l, 24, generator=g, dtype=torch.float64) / 4
        y = torch.where(torch.rand(l, generator=g) < 0.3, 1.0, -1.0).to(torch.float64)
        c = torch.where(y > 0, 1.7, 0.6).to(torch.float64)
        lo, hi = rank * l // world, (rank + 1) * l // world
        probs.append((Phi[lo:hi].contiguous(), y[lo:hi].contiguous(), c[lo:hi].contiguous()))
    sl._Red.STATS.update(rccl=0, peer=0)
    single = [sl.ipm_svc_dual(P, y, c, group=group) for P, y, c in probs]
    n_single = sl._Red.STATS["rccl"]
    sl._Red.STATS.update(rccl=0, peer=0)
    batched = sl._drive([sl._ipm_gen(P, y, c) for P, y, c in probs], sl._Red(group))
    n_batch = sl._Red.STATS["rccl"]
    da = max(float((a1 - a2).abs().max()) for (a1, _, _), (a2, _, _) in zip(single, batched))
    drho = max(abs(r1 - r2) for (_, r1, _), (_, r2, _) in zip(single, batched))
    t = torch.tensor([da, drho], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    iters = [it for _, _, it in single]
    assert iters == [it for _, _, it in batched]
    return float(t[0]), float(t[1]), n_single, n_batch, iters


@pytest.mark.parametrize("world", [2, 4])
def test_batched_ipm_one_collective_per_step(world):
    """the row-sharded interior points of one SVC fit run in lock-step from one host
    thread (svc_lowrank._drive) — the same iterates as solving them one after another (≤ 1e-8; the
    reductions are the same sums, merged into one buffer), with the collectives per iteration
    counted per FIT (≤ 17 + the 3 setup reductions), not per problem."""
    da, drho, n_single, n_batch, iters = _run("_ipm_batched", world)
    assert da <= 1e-8 and drho <= 1e-8, (da, drho)
    assert n_batch <= 17 * max(iters) + 3, (n_batch, iters)
    assert n_single >= 2 * n_batch, (n_single, n_batch)

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
    from hfens.models import logreg_solver
    assert logreg_solver.LAST_PATH["path"] == "fused"   # the one-launch kernel ran
    for a, b in zip(mh, md):
        assert torch.allclose(a.coef_, b.coef_.cpu(), atol=1e-6)
        assert torch.allclose(a.intercept_, b.intercept_.cpu(), atol=1e-6)


@pytest.mark.parametrize("pen", ["l1", "l2"])
def test_logreg_fused_matches_device_loop(dev, monkeypatch, pen):
    """logreg_fused (one launch, per-model stopping) reaches the same optimum as the host-driven
    device loop (the data-parallel path) on the stacking shape: 6 masks, 17 features."""
    from hfens.models import logreg_solver
    X, y = _data(8000, 17, 17)
    masks = torch.ones(6, 8000, dtype=torch.bool)
    for k in range(5):
        masks[k, k::5] = False
    kw = dict(penalty=pen, solver="liblinear" if pen == "l1" else "lbfgs", class_weight="balanced")
    out = {}
    for fused in (False, True):
        monkeypatch.setattr(logreg_solver, "FUSED", fused)
        ms = [LogisticRegression(**kw) for _ in range(6)]
        fit_logreg_batch(ms, X.to(dev), y.to(dev), masks.to(dev))
        out[fused] = ms
    for a, b in zip(out[False], out[True]):
        assert torch.allclose(a.coef_, b.coef_, atol=1e-7)
        assert torch.allclose(a.intercept_, b.intercept_, atol=1e-7)


@pytest.mark.parametrize("refit", [False, True])
def test_logreg_preset_matches_finish(dev, refit):
    """launch_logreg_batch(prep=..., preset=True) (the stacking fit's meta model: set_fitted at
    launch, behind the enqueued solve) leaves the same fitted models as set_fitted at finish; after a
    cooperative-exchange fallback (simulated: ``refit``) the models are set again from the re-solve."""
    from hfens.models import logreg_solver
    X, y = _data(4000, 3, 29)
    Xd, yd = X.to(dev).to(torch.float64), y.to(dev).to(torch.float64)
    out = []
    for preset in (False, True):
        ms = [LogisticRegression()]
        prep = logreg_solver.logreg_label_prep(ms, yd, Xd.shape[0], Xd.device)
        h = logreg_solver.launch_logreg_batch(ms, Xd, yd, prep=prep, preset=preset)
        assert h.get("preset", False) == preset
        if refit and preset:
            ms[0].intercept_.fill_(123.0)      # (what a stale launch-time copy would leave)
            h["fused"]["refit"] = True
        logreg_solver.finish_logreg_batch(h)
        out.append(ms[0])
    assert torch.equal(out[0].coef_, out[1].coef_)
    assert torch.equal(out[0].intercept_, out[1].intercept_)
    assert torch.equal(out[0].n_iter_, out[1].n_iter_)


@pytest.mark.parametrize("pen,n,members", [("l1", 8000, 5), ("l2", 10007, 16), ("l1", 300, 3), ("l2", 2000, 1)])
def test_logreg_coop_matches_single_workgroup(dev, monkeypatch, pen, n, members):
    """logreg_coop (members exchange ordered partial sums of H, g and the line-search losses) takes
    the same Newton steps as the one-workgroup kernel up to summation order; members=1 is the
    one-workgroup kernel itself.  Also a model with fewer rows than members×1024 threads."""
    from hfens.models import logreg_solver
    X, y = _data(n, 17, 23)
    B = 6 if pen == "l1" else 1
    masks = torch.ones(B, n, dtype=torch.bool)
    for k in range(min(B, 5)):
        masks[k, k::5] = False
    kw = dict(penalty=pen, solver="liblinear" if pen == "l1" else "lbfgs", class_weight="balanced")
    out = {}
    for m in (1, members):
        monkeypatch.setattr(logreg_solver, "MEMBERS", m)
        ms = [LogisticRegression(**kw) for _ in range(B)]
        fit_logreg_batch(ms, X.to(dev), y.to(dev), masks.to(dev))
        assert logreg_solver.LAST_PATH["members"] == min(m, 256 // B)
        assert not logreg_solver.LAST_PATH.get("coop_fallback")
        out[m] = ms
    for a, b in zip(out[1], out[members]):
        # both stop at the solver tolerance (the fused-vs-loop test's 1e-7)
        d = float((a.coef_ - b.coef_).abs().max())
        assert d < 1e-7, d
        assert torch.allclose(a.intercept_, b.intercept_, atol=1e-7)


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


@pytest.mark.parametrize("subsample", [1.0, 0.7])
def test_gbdt_stump_paths_bit_identical(dev, monkeypatch, subsample):
    """The three depth-1 device paths — launch-per-step, gbdt_stumps_fused (one launch, one
    workgroup per model) and gbdt_stump_stage (one launch per stage over row tiles × models) —
    produce the same trees bit for bit: features, thresholds, leaf values, impurities,
    node weights, train_score_."""
    from hfens.models import hist_gbdt
    monkeypatch.setattr(hist_gbdt, "SKLEARN_TIES", False)
    X, y = _data(6000, 17, 51)
    masks = torch.ones(6, 6000, dtype=torch.bool)
    for k in range(5):
        masks[k, k::5] = False
    out = {}
    for path in ("launch", "fused", "stage"):
        monkeypatch.setattr(hist_gbdt, "STUMP_PATH", path)
        monkeypatch.setattr(hist_gbdt, "FUSED_STUMPS", path == "fused")
        ms = [GradientBoostingClassifier(n_estimators=60, max_depth=1, subsample=subsample, random_state=s)
              for s in range(6)]
        fit_gbdt_batch(ms, X.to(dev), y.to(dev), masks.to(dev))
        assert hist_gbdt.LAST_PATH["path"] == path
        out[path] = ms
    for other in ("fused", "stage"):
        for a, b in zip(out["launch"], out[other]):
            for attr in ("tree_feature_", "tree_threshold_", "tree_value_", "tree_impurity_",
                         "tree_weighted_n_node_samples_", "train_score_"):
                assert torch.equal(getattr(a, attr), getattr(b, attr)), (other, attr)


@pytest.mark.parametrize("rows,subsample", [(6000, 1.0), (150000, 0.7)])
def test_gbdt_stage_mfma_hist_bit_identical(dev, monkeypatch, rows, subsample):
    """gbdt_stump_stage with the i8-MFMA histogram (binary and <= 8-bin features as 7-bit slice
    GEMMs, HFENS_GBDT_MFMA=1) equals the int64 VALU histogram (=0) bit for bit; the data mixes
    binary, 3- to 6-bin ordinal, constant and wide continuous features, and 150k rows spread each
    model over many workgroups and sub-tiles."""
    from hfens.models import hist_gbdt
    monkeypatch.setattr(hist_gbdt, "STUMP_PATH", "stage")
    monkeypatch.setattr(hist_gbdt, "FUSED_STUMPS", False)
    X, y = _data(rows, 24, 53)
    g = torch.Generator().manual_seed(5)
    X[:, 4] = torch.randint(0, 3, (rows,), generator=g).double()
    X[:, 5] = torch.randint(0, 6, (rows,), generator=g).double() * 0.5
    X[:, 7] = 1.0
    masks = torch.ones(3, rows, dtype=torch.bool)
    masks[1, ::4] = False
    masks[2, 1::3] = False
    out = {}
    for mf, nt in (("0", "512"), ("1", "512"), ("1", "1024")):
        monkeypatch.setenv("HFENS_GBDT_MFMA", mf)
        monkeypatch.setenv("HFENS_SG_THREADS", nt)
        ms = [GradientBoostingClassifier(n_estimators=40, max_depth=1, subsample=subsample, random_state=s)
              for s in range(3)]
        fit_gbdt_batch(ms, X.to(dev), y.to(dev), masks.to(dev))
        assert hist_gbdt.LAST_PATH["path"] == "stage"
        out[mf + nt] = ms
    for key in ("1512", "11024"):
        for a, b in zip(out["0512"], out[key]):
            for attr in ("tree_feature_", "tree_threshold_", "tree_value_", "tree_impurity_",
                         "tree_weighted_n_node_samples_", "train_score_"):
                assert torch.equal(getattr(a, attr), getattr(b, attr)), (key, attr)


@pytest.mark.parametrize("rows", [2500, 70000])
def test_gbdt_stage_sklearn_ties_match_host(dev, rows):
    """gbdt_stump_stage with sklearn's feature-visit tie-break (duplicated columns force exact
    gain ties) equals the host mirror, which visits features in the same order; large row counts
    spread each model over many workgroups."""
    from hfens.models import hist_gbdt
    X, y = _data(rows, 12, 52)
    X[:, 6] = X[:, 3] + 1.0
    X[:, 9] = 2.0 * X[:, 2]
    mh = [GradientBoostingClassifier(n_estimators=40, max_depth=1, random_state=s) for s in (2020, 7)]
    md = [GradientBoostingClassifier(n_estimators=40, max_depth=1, random_state=s) for s in (2020, 7)]
    fit_gbdt_batch(mh, X, y)
    fit_gbdt_batch(md, X.to(dev), y.to(dev))
    assert hist_gbdt.LAST_PATH["path"] == "stage"
    for a, b in zip(mh, md):
        assert torch.equal(a.tree_feature_, b.tree_feature_.cpu())
        assert torch.equal(a.tree_threshold_, b.tree_threshold_.cpu())
        assert torch.allclose(a.tree_value_, b.tree_value_.cpu(), rtol=1e-12, atol=1e-15)
        assert torch.allclose(a.train_score_, b.train_score_.cpu(), rtol=1e-12)


def _dp_stage_worker(rank, world, port, q, xgmi="0", T=30, subsample=1.0, fail_open_rank=-1, env=None):
    import os
    # ranks sharing ONE card: one hardware queue each, so 4 processes' queues are all resident
    # (a spinning peer kernel must not keep another rank's queue from being scheduled)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HFENS_XGMI=xgmi, GPU_MAX_HW_QUEUES="1")
    os.environ.update(env or {})
    import torch.distributed as dist
    from hfens.models import hist_gbdt
    from hfens.parallel import dist as pdist
    from hfens.parallel.dist import shard_rows
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        if rank == fail_open_rank:   # this rank cannot map its peers' buffers
            from hfens import ops

            def _no_map(*a):
                raise RuntimeError("injected: hipIpcOpenMemHandle failed")
            setattr(ops.ext(), "xgmi_ipc_open", _no_map)
        X, y = _data(9000, 17, 53)
        for _ in range(2):   # twice: the second fit reuses the peer buffers (epochs continue)
            ms = [GradientBoostingClassifier(n_estimators=T, max_depth=1, subsample=subsample, random_state=s)
                  for s in (1, 2)]
            fit_gbdt_batch(ms, shard_rows(X, rank, world).to(dev), shard_rows(y, rank, world).to(dev),
                           group=dist.group.WORLD)
        if rank == 0:
            from hfens.parallel import xgmi as _xg
            q.put((hist_gbdt.LAST_PATH["path"], hist_gbdt.COLLECTIVES["per_stage"],
                   hist_gbdt.COLLECTIVES.get("xgmi_per_stage", 0.0), hist_gbdt.GRAPH_INFO.get("units", 0),
                   [(m.tree_feature_.cpu().numpy(), m.tree_threshold_.cpu().numpy(), m.tree_value_.cpu().numpy(),
                     m.tree_impurity_.cpu().numpy(), m.train_score_.cpu().numpy()) for m in ms],
                   list(_xg.PROBES.values()), list(hist_gbdt.GRAPH_PROBES.values())))
    finally:
        pdist.shutdown()


def _run_dp_stage(world, xgmi, T=30, subsample=1.0, fail_open_rank=-1, env=None, probes=False):
    import socket
    import torch.multiprocessing as mp
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_stage_worker, args=(r, world, port, q, xgmi, T, subsample, fail_open_rank, env))
             for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=150)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out if probes else out[:5]


def _check_dp_stage_equal(dev, got, T=30, subsample=1.0):
    X, y = _data(9000, 17, 53)
    ms = [GradientBoostingClassifier(n_estimators=T, max_depth=1, subsample=subsample, random_state=s) for s in (1, 2)]
    fit_gbdt_batch(ms, X.to(dev), y.to(dev))
    for (f, t, v, imp, ts), m in zip(got, ms):
        assert np.array_equal(f, m.tree_feature_.cpu().numpy())
        assert np.array_equal(t, m.tree_threshold_.cpu().numpy())
        assert np.array_equal(v, m.tree_value_.cpu().numpy())
        assert np.array_equal(imp, m.tree_impurity_.cpu().numpy())
        assert np.array_equal(ts, m.train_score_.cpu().numpy())


def test_gbdt_stage_data_parallel_bit_identical(dev):
    """Two ranks on the card, RCCL-free gloo group with the peer path off (HFENS_XGMI=0): the
    sharded stage path issues exactly ONE collective per boosting stage and reproduces the
    single-process fit bit for bit, impurities included."""
    path, per_stage, xg, units, got = _run_dp_stage(2, "0")
    assert path == "stage" and per_stage == 1.0 and xg == 0.0
    _check_dp_stage_equal(dev, got)


@pytest.mark.parametrize("world,subsample", [(2, 1.0), (4, 1.0), (4, 0.8)])
def test_gbdt_stage_xgmi_bit_identical(dev, world, subsample):
    """the per-stage sum through IPC-mapped peer buffers (parallel/xgmi.py, one
    kernel per stage, captured in the stage graph) — 2 and 4 processes on one card, each mapping
    the others' buffers — gives the single-process fit bit for bit with ZERO collectives per
    stage (the process group only exchanged the IPC handles)."""
    path, per_stage, xg, units, got = _run_dp_stage(world, "1", subsample=subsample)
    assert path == "stage" and per_stage == 0.0 and xg == 1.0
    assert units == 31 // 3          # the stage loop ran as replayed HIP graphs
    _check_dp_stage_equal(dev, got, subsample=subsample)


def test_xgmi_first_use_probe_validates(dev):
    """the first use of the peer buffers runs probe reductions (int64 sum over several
    chunks, f64 sum / max / min in rank order) through the peer kernel and through the collective
    library, bit for bit, and the first stage-graph use replays captured reductions against eager
    ones — both pass on every rank, so the fit keeps the peer kernel inside the replayed graph."""
    path, per_stage, xg, units, got, pr, gpr = _run_dp_stage(2, "try", probes=True)
    assert pr and all(p["ok"] and not p["mismatches"] for p in pr), pr
    assert gpr and all(p["ok"] and p["peer"] for p in gpr), gpr
    assert per_stage == 0.0 and xg == 1.0 and units == 31 // 3
    _check_dp_stage_equal(dev, got)


def test_xgmi_probe_mismatch_falls_back_together(dev):
    """One rank's probe result disagrees with the library's (HFENS_XGMI_PROBE_CORRUPT): every rank
    drops the peer path together, the mismatch is recorded with the rank that saw it, and the fit
    runs on the collective library — one all-reduce per stage, the single-process model bit for bit."""
    path, per_stage, xg, units, got, pr, gpr = _run_dp_stage(3, "try", env={"HFENS_XGMI_PROBE_CORRUPT": "1"},
                                                             probes=True)
    assert len(pr) == 1 and not pr[0]["ok"] and any(m.startswith("rank 1:") for m in pr[0]["mismatches"]), pr
    assert path == "stage" and per_stage == 1.0 and xg == 0.0
    _check_dp_stage_equal(dev, got)


def test_xgmi_probe_local_raise_falls_back_together(dev):
    """one rank RAISES inside the peer-probe's local phase (HFENS_XGMI_PROBE_RAISE) and
    so never runs its peer kernels: the others' peer waits time out, every rank still issues the
    same collective sequence (no hang), all drop the peer path together and the fit runs on the
    collective library, bit for bit."""
    path, per_stage, xg, units, got, pr, gpr = _run_dp_stage(
        2, "try", env={"HFENS_XGMI_PROBE_RAISE": "1", "HFENS_XGMI_TIMEOUT": "2"}, probes=True)
    assert len(pr) == 1 and not pr[0]["ok"] and any(m.startswith("rank 1:") for m in pr[0]["mismatches"]), pr
    assert path == "stage" and per_stage == 1.0 and xg == 0.0
    _check_dp_stage_equal(dev, got)


def test_stage_graph_probe_local_raise_runs_eagerly(dev):
    """one rank's stage-graph capture raises (HFENS_GBDT_GRAPH_PROBE_RAISE): nobody
    replays (the capture agreement comes first), every rank runs the stage loop eagerly on the
    still-valid peer kernel, bit for bit."""
    path, per_stage, xg, units, got, pr, gpr = _run_dp_stage(2, "1", env={"HFENS_GBDT_GRAPH_PROBE_RAISE": "0"},
                                                             probes=True)
    assert pr and pr[0]["ok"]
    assert gpr and not gpr[0]["ok"] and any(m.startswith("rank 0:") for m in gpr[0]["mismatches"]), gpr
    assert units == 0 and per_stage == 0.0 and xg == 1.0
    _check_dp_stage_equal(dev, got)


def test_stage_graph_probe_mismatch_runs_eagerly(dev):
    """The stage-graph probe disagrees on one rank (HFENS_GBDT_GRAPH_PROBE_CORRUPT): every rank runs
    the stage loop eagerly (no replayed units) on the still-valid peer kernel, bit for bit."""
    path, per_stage, xg, units, got, pr, gpr = _run_dp_stage(2, "1", env={"HFENS_GBDT_GRAPH_PROBE_CORRUPT": "1"},
                                                             probes=True)
    assert pr and pr[0]["ok"]
    assert gpr and not gpr[0]["ok"] and gpr[0]["mismatches"], gpr
    assert units == 0 and per_stage == 0.0 and xg == 1.0
    _check_dp_stage_equal(dev, got)


def test_gbdt_stage_xgmi_mapping_failure_falls_back(dev):
    """HFENS_XGMI=try and ONE rank cannot map a peer's buffer: every rank drops the peer path
    together (the mapping errors are gathered before anyone uses the kernel) and the group keeps the
    collective path — one all-reduce per stage, the single-process fit bit for bit, no hang."""
    path, per_stage, xg, units, got = _run_dp_stage(3, "try", fail_open_rank=1)
    assert path == "stage" and per_stage == 1.0 and xg == 0.0
    _check_dp_stage_equal(dev, got)


def _gbdt_outputs(ms):
    return [(m.tree_feature_.cpu().numpy(), m.tree_threshold_.cpu().numpy(), m.tree_value_.cpu().numpy(),
             m.tree_impurity_.cpu().numpy(), m.train_score_.cpu().numpy()) for m in ms]


@pytest.mark.parametrize("T,subsample", [(20, 1.0), (100, 0.8)])
def test_gbdt_stage_graph_bit_identical(dev, monkeypatch, T, subsample):
    """The HIP-graph stage loop (3-stage units replayed with a device stage counter) gives the
    eager loop's model bit for bit."""
    from hfens.models import hist_gbdt
    X, y = _data(20000, 17, 61)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(hist_gbdt, "STAGE_GRAPH", mode)
        ms = [GradientBoostingClassifier(n_estimators=T, max_depth=1, subsample=subsample, random_state=s)
              for s in (3, 4)]
        fit_gbdt_batch(ms, X.to(dev), y.to(dev))
        assert hist_gbdt.LAST_PATH["path"] == "stage"
        assert hist_gbdt.GRAPH_INFO["units"] == (0 if mode == "0" else (T + 1) // 3)
        out[mode] = _gbdt_outputs(ms)
    for a, b in zip(out["0"], out["1"]):
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_gbdt_stage_graph_rccl_world1(dev, monkeypatch):
    """The RCCL branch (backend "nccl", peer-memory path off) on a one-rank group: its per-stage
    all-reduces are captured in the stage graph, one collective per stage, and the model equals the
    single-process fit."""
    import tempfile
    import torch.distributed as dist
    from hfens.models import hist_gbdt
    from hfens.parallel import xgmi
    monkeypatch.setattr(xgmi, "MODE", "0")
    store = tempfile.mktemp(prefix="hfens_pg_")   # file store: no TCP port to race for
    dist.init_process_group("nccl", init_method=f"file://{store}", rank=0, world_size=1,
                            device_id=torch.device(dev))
    try:
        g = dist.new_group([0], backend="nccl")
        X, y = _data(9000, 17, 53)
        ms = [GradientBoostingClassifier(n_estimators=30, max_depth=1, random_state=s) for s in (1, 2)]
        fit_gbdt_batch(ms, X.to(dev), y.to(dev), group=g)
        assert hist_gbdt.LAST_PATH["path"] == "stage" and hist_gbdt.COLLECTIVES["per_stage"] == 1.0
        assert hist_gbdt.GRAPH_INFO["units"] == 31 // 3
        got = _gbdt_outputs(ms)
    finally:
        dist.destroy_process_group()
    ref = [GradientBoostingClassifier(n_estimators=30, max_depth=1, random_state=s) for s in (1, 2)]
    fit_gbdt_batch(ref, X.to(dev), y.to(dev))
    for a, b in zip(got, _gbdt_outputs(ref)):
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


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


@pytest.mark.parametrize("otf", [True, False])
@pytest.mark.parametrize("rows,slice_", [(2500, 384), (6000, 384), (6000, 1024), (6000, 2048)])
def test_smo_coop_matches_single_workgroup(dev, monkeypatch, rows, slice_, otf):
    """The cooperative SMO (W workgroups per problem, in-launch exchanges) follows the same pair
    sequence as the one-workgroup kernel: identical iteration counts and support sets, α and ρ equal
    to accumulated rounding (the members sum ρ's free-vector average in a different order)."""
    from hfens.models import smo
    X, y = _data(rows, 17, 21)
    Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).to(dev)
    yd = y.to(dev)
    Zs, ys = [Z[: rows * 4 // 5], Z], [yd[: rows * 4 // 5], yd]

    monkeypatch.setattr(smo, "SOLVER", "exact")
    monkeypatch.setattr(smo, "COOP_OTF", otf)   # Gram rows recomputed per pair vs read from the stored Gram

    def fit(coop):
        monkeypatch.setattr(smo, "COOP", coop)
        monkeypatch.setattr(smo, "COOP_MIN_SLICE", slice_)
        svcs = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in Zs]
        smo.fit_svc_batch(svcs, Zs, ys)
        return svcs, dict(smo.LAST_SMO_INFO)

    one, info1 = fit(False)
    many, info2 = fit(True)
    assert info1["members"] == 1 and info2["members"] > 1
    otf_fits = -(-info2["max_l"] // info2["members"]) <= smo._OTF_MAX_S   # register tile without spills
    assert info2["solver"] == ("coop-otf" if otf and otf_fits else "coop")
    for a, b in zip(one, many):
        assert a.n_iter_ == b.n_iter_
        assert torch.equal(a.support_, b.support_)
        # same pairs in the same order; α agree to accumulated rounding (≤ 1e-13 measured)
        assert torch.allclose(a._dual_coef_, b._dual_coef_, rtol=1e-10, atol=1e-12)
        assert float(a._intercept_[0]) == pytest.approx(float(b._intercept_[0]), rel=1e-10, abs=1e-12)
        # Platt's Newton fit stops at |∇| < 1e-5, so rounding-level decision values move A, B by ~1e-6
        assert a._probA.item() == pytest.approx(b._probA.item(), rel=1e-4)
        assert a._probB.item() == pytest.approx(b._probB.item(), rel=1e-4, abs=1e-5)


def test_quantize_bins_kernel_matches_searchsorted(dev):
    """K7 quantize_bins (LDS edge table, binary search) = torch.searchsorted on the same edges,
    for f64 and f32 rows, values on and between edges, above the last edge."""
    from hfens.models.binning import fit_bins
    X, _ = _data(70000, 30, 91)
    X[:, 3] = torch.round(X[:, 3] * 2)
    bm = fit_bins(X.to(dev), 256)
    Xn, _ = _data(5000, 30, 92)
    Xn[:7, :] = 1e9
    for Z in (Xn.to(dev), Xn.to(dev).float()):
        got = bm.transform(Z)
        X32 = Z.to(torch.float32).t().contiguous()
        ref = torch.searchsorted(bm.edges, X32)
        ref = torch.minimum(ref, (bm.nbins.to(ref.dtype) - 1)[:, None]).to(torch.uint8)
        assert torch.equal(got, ref)


def test_scaler_batch_matches_per_fold_scalers(dev):
    """K2: the native batched fold scalers (mean / population variance / scaled rows of every
    fold subset in one pass) equal StandardScaler fitted per fold."""
    from hfens.models.scaler import StandardScaler
    from hfens.models.stack_trainer import scaler_batch_device
    X, _ = _data(9001, 17, 91)
    X[:, 3] = 2.0                                   # a constant column: scale 1
    Xd = X.to(dev)
    rng = np.random.default_rng(3)
    folds = rng.integers(0, 5, 9001)
    rows = [np.nonzero(folds != k)[0] for k in range(5)] + [np.arange(9001)]
    mean, var, Z, offs, _ = scaler_batch_device(Xd, rows)
    for k, r in enumerate(rows):
        sc = StandardScaler().fit(Xd[torch.as_tensor(r, device=dev)])
        assert torch.allclose(mean[k], sc.mean_, rtol=1e-13, atol=1e-13)
        assert torch.allclose(var[k], sc.var_, rtol=1e-11, atol=1e-13)
        Zk = sc.transform(Xd[torch.as_tensor(r, device=dev)])
        dz = (Z[offs[k]:offs[k + 1]] - Zk).abs().max(0).values
        assert float(dz.max()) < 1e-11, (k, dz.tolist(), sc.scale_.tolist())
        # the constant column: exact mean, variance 0, scale 1 (sklearn 0.23.2), in both paths
        assert float(var[k, 3]) == 0.0 and float(sc.var_[3]) == 0.0
    assert torch.all(Z[:, 3] == 0)


@pytest.mark.parametrize("rows", [2500, 6000])
def test_smo_shared_gram_matches_own_grams(dev, monkeypatch, rows):
    """Platt sub-problems reading their fit's final-problem Gram through a column map
    (smo_coop_kernel<K4, true>) take the same pairs as with Grams of their own: identical iteration
    counts and α of EVERY problem (the Platt ones included), ρ to its member-sum order."""
    from hfens.models import smo
    X, y = _data(rows, 17, 23)
    Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).to(dev)
    yd = y.to(dev)
    Zs, ys = [Z[: rows * 4 // 5], Z], [yd[: rows * 4 // 5], yd]
    monkeypatch.setattr(smo, "SOLVER", "exact")
    monkeypatch.setattr(smo, "COOP_OTF", False)
    monkeypatch.setattr(smo, "COOP_MIN_SLICE", 384)

    def run(share):
        monkeypatch.setattr(smo, "SHARE_GRAM", share)
        svcs = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in Zs]
        st = smo.launch_svc_batch(svcs, Zs, ys)
        res = [(p.fit, p.fold, st["sol"][id(p)]) for p in st["all_probs"] if p.rows is not None]
        res = [(f, k, a.cpu().clone(), float(r), int(it)) for f, k, (a, r, it) in res]
        info = dict(smo.LAST_SMO_INFO)
        smo.finish_svc_batch(st)
        return res, info, svcs

    own, i_own, s_own = run(False)
    sh, i_sh, s_sh = run(True)
    assert i_own["members"] > 1 and i_own["grams"] == 12 and i_sh["grams"] == 2
    for (f, k, a, r, it), (f2, k2, b, r2, it2) in zip(own, sh):
        assert (f, k, it) == (f2, k2, it2)
        assert torch.equal(a, b)
        assert r == pytest.approx(r2, rel=1e-12, abs=1e-14)
    for a, b in zip(s_own, s_sh):
        assert torch.equal(a.support_, b.support_)
        assert a._probA.item() == pytest.approx(b._probA.item(), rel=1e-9)
        assert a._probB.item() == pytest.approx(b._probB.item(), rel=1e-9, abs=1e-12)


def test_develop_plan_ahead_identical(dev, monkeypatch):
    """The stacking bookkeeping computed under the LassoCV path (folds, SVC problem expansions,
    Platt column maps: pipeline.PLAN_AHEAD) gives the same fit as computing it in line."""
    from hfens import pipeline
    from hfens.io.synth import make_hf_cohort
    from hfens.models import stack_trainer
    # (the SVC batch launched from the host selection in both: the prelaunched batch computes γ on
    # the device, last-bit different — test_prelaunched_svc_batch_matches)
    monkeypatch.setattr(stack_trainer, "PRELAUNCH_SVC", False)
    Xd, yd, names = make_hf_cohort(3000, 40, seed=77, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(1000, 40, seed=78, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    out = {}
    for ahead in (False, True):
        monkeypatch.setattr(pipeline, "PLAN_AHEAD", ahead)
        r = pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev)
        out[ahead] = r
    assert np.array_equal(out[False].selected, out[True].selected)
    assert torch.equal(out[False].proba_sel, out[True].proba_sel)
    m0, m1 = out[False].model, out[True].model
    assert torch.equal(m0.oof_meta_, m1.oof_meta_)


@pytest.mark.parametrize("wgs,atomic", [("1", None), ("2", None), ("4", None), ("1", "16"), ("2", "16"),
                                         ("4", "16")])
def test_gbdt_stage_plan_sizes_partials(dev, monkeypatch, wgs, atomic):
    """the partial-slot buffer is sized from the kernel's own launch plan
    (gbdt_stage_plan), so every workgroups-per-CU setting and model count runs (no 'partials
    buffer too small'), and the trees do not depend on the grid.  atomic = None: every workgroup
    adds into the slot with int64 atomics (the default); "16": above 16 workgroups per model the
    partial slots + reduce launch — the same integers either way."""
    from hfens.models import hist_gbdt
    X, y = _data(120_000, 12, 7)
    ref = None
    monkeypatch.setenv("HFENS_SG_WGS_PER_CU", wgs)
    if atomic is not None:
        monkeypatch.setenv("HFENS_SG_ATOMIC_GROUPS", atomic)
    for B in (1, 5, 6):
        ms = [GradientBoostingClassifier(n_estimators=4, max_depth=1, random_state=s) for s in range(B)]
        fit_gbdt_batch(ms, X.to(dev), y.to(dev))
        assert hist_gbdt.LAST_PATH["path"] == "stage"
        plan = hist_gbdt.stage_plan(X.shape[0], B, int(ms[0]._bin_mapper.nb_host.sum()),
                                    torch.cuda.get_device_properties(dev).multi_processor_count)
        assert plan[1] * plan[0] >= X.shape[0] and (plan[2] == 0) == (plan[3] == 0)
        assert plan[2] == (1 if atomic is not None and plan[1] > int(atomic) else 0)
        if B == 1:
            ref = (ms[0].tree_feature_.cpu(), ms[0].tree_value_.cpu(), ms[0].train_score_.cpu())
        assert torch.equal(ms[0].tree_feature_.cpu(), ref[0])
        assert torch.equal(ms[0].tree_value_.cpu(), ref[1])
        assert torch.equal(ms[0].train_score_.cpu(), ref[2])


def _lowrank_dp_worker(rank, world, port, q, xgmi="0"):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GPU_MAX_HW_QUEUES="1", HFENS_XGMI=xgmi)
    import torch.distributed as dist
    from hfens.models import svc_lowrank
    from hfens.parallel import dist as pdist
    from hfens.parallel.dist import shard_rows
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        Z, y = _data(6000, 8, 71)
        svc = SVC(class_weight="balanced", probability=True, random_state=2020)
        svc_lowrank.fit_svc_lowrank_batch([svc], [shard_rows(Z, rank, world).to(dev)],
                                          [shard_rows(y, rank, world).to(dev)], n_landmarks=256,
                                          group=dist.group.WORLD)
        if rank == 0:
            q.put((svc._dual_coef_.cpu(), float(svc._intercept_[0]), svc._probA.item(), svc._probB.item(),
                   svc.support_.cpu(), svc_lowrank.LAST_INFO["row_sharded"], dict(svc_lowrank._Red.STATS)))
    finally:
        from hfens.parallel import xgmi as _xg
        _xg.release_all()
        pdist.shutdown()


@pytest.mark.parametrize("world,xgmi", [(2, "0"), (4, "0"), (2, "1"), (4, "1")])
def test_lowrank_svc_row_sharded_threads(dev, world, xgmi):
    """the row-sharded interior point with its concurrent Platt-CV solves (3
    host threads + the final solve, each on its own stream AND its own communicator) — 2 / 4
    processes on one card over gloo — equals the one-process GPU fit to 1e-8.  xgmi = "1" (VERDICT
    r3 next #5): every reduction of the solves is one peer-memory f64 kernel folding the ranks in
    rank order (parallel/xgmi.py reduce_f64_) — ZERO collectives inside the interior point — with
    the solves run from one thread (svc_lowrank._threads_safe)."""
    import socket
    import torch.multiprocessing as mp
    from hfens.models import svc_lowrank
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_lowrank_dp_worker, args=(r, world, port, q, xgmi)) for r in range(world)]
    for p in procs:
        p.start()
    coef, ic, pa, pb, sup, sharded, red = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    Z, y = _data(6000, 8, 71)
    ref = SVC(class_weight="balanced", probability=True, random_state=2020)
    svc_lowrank.fit_svc_lowrank_batch([ref], [Z.to(dev)], [y.to(dev)], n_landmarks=256)
    assert sharded is True
    if xgmi == "1":
        assert red["rccl"] == 0 and red["peer"] > 0, red
    else:
        assert red["peer"] == 0 and red["rccl"] > 0, red
    assert torch.equal(sup, ref.support_.cpu())
    assert torch.allclose(coef, ref._dual_coef_.cpu(), rtol=0, atol=1e-8)
    assert abs(ic - float(ref._intercept_[0])) < 1e-8
    # Platt's Newton stops at |grad| < 1e-5: decision values equal to ~1e-12 move (A, B) by ~1e-8
    assert abs(pa - ref._probA.item()) < 1e-6 and abs(pb - ref._probB.item()) < 1e-6


@pytest.mark.parametrize("otf", [False, True])
def test_smo_coop_late_member_falls_back(dev, monkeypatch, otf):
    """a member that arrives late (HFENS_SMO_INJECT_DELAY_MS holds member 1 of
    problem 0 back) makes the others give up at the exchange deadline (HFENS_SMO_WAIT_MS) instead
    of spinning for seconds; the launch reports smo_err, the batch is re-solved by the
    one-workgroup kernel, and the model equals the one-workgroup fit.  The timeout's own cost —
    the faulted fit minus the one-workgroup fit minus the injected delay — stays ≤ 50 ms."""
    import time
    import warnings
    from hfens.models import smo
    rows = 3000
    X, y = _data(rows, 17, 23)
    Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).to(dev)
    yd = y.to(dev)
    Zs, ys = [Z[: rows * 4 // 5], Z], [yd[: rows * 4 // 5], yd]
    monkeypatch.setattr(smo, "SOLVER", "exact")
    monkeypatch.setattr(smo, "COOP_OTF", otf)
    monkeypatch.setenv("HFENS_SMO_WAIT_MS", "20")
    assert smo.coop_resident(dev) >= torch.cuda.get_device_properties(dev).multi_processor_count

    def fit(coop, delay_ms=None):
        monkeypatch.setattr(smo, "COOP", coop)
        if delay_ms is None:
            monkeypatch.delenv("HFENS_SMO_INJECT_DELAY_MS", raising=False)
        else:
            monkeypatch.setenv("HFENS_SMO_INJECT_DELAY_MS", str(delay_ms))
        svcs = [SVC(class_weight="balanced", probability=True, random_state=2020) for _ in Zs]
        torch.cuda.synchronize()
        t = time.perf_counter()
        with warnings.catch_warnings(record=True) as wl:
            warnings.simplefilter("always")
            smo.fit_svc_batch(svcs, Zs, ys)
        torch.cuda.synchronize()
        return svcs, dict(smo.LAST_SMO_INFO), 1e3 * (time.perf_counter() - t), wl

    fit(False)                                             # warm-up (kernels loaded)
    one, info1, t_one, _ = fit(False)
    fb, info2, t_fb, wl = fit(True, delay_ms=60)
    assert info1["members"] == 1
    assert info2.get("coop_fallback") is True and any("timed out" in str(w.message) for w in wl)
    for a, b in zip(one, fb):
        assert a.n_iter_ == b.n_iter_
        assert torch.equal(a.support_, b.support_)
        assert torch.equal(a._dual_coef_, b._dual_coef_)
    assert t_fb - t_one - 60.0 <= 50.0, (t_fb, t_one)
    ok, info3, _, wl3 = fit(True)                          # no injection: no fallback
    assert not info3.get("coop_fallback") and info3["members"] > 1 and not wl3


def test_device_svc_oof_matches_fold_models(dev, monkeypatch):
    """The stacking trainer's SVC out-of-fold column computed on the device behind the SMO
    (smo.enqueue_svc_oof: decision sums over the final problems' rows, Platt sigmoid + coupling from
    the device (A, B)) equals the fold models' predict_proba up to the decision sums' f32 rounding:
    the batched kernel sums 1024-point f32 partials in f64 over every point of the problem, the
    fold model's rbf_decision one f32 sum over its support vectors (measured max |Δp| 5e-5, typical
    1e-6), and the meta model fitted on it predicts the same probabilities to that order."""
    from hfens import pipeline
    from hfens.models import stack_trainer
    from hfens.io.synth import make_hf_cohort
    Xd, yd, names = make_hf_cohort(3000, 40, seed=91, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(1000, 40, seed=92, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(stack_trainer, "DEVICE_SVC_OOF", flag)
        out[flag] = pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev)
    m0, m1 = out[False].model, out[True].model
    d = (m0.oof_meta_ - m1.oof_meta_).abs()
    assert float(d[:, 1:].max()) == 0.0            # the other columns are untouched
    assert float(d[:, 0].max()) <= 2e-4, float(d[:, 0].max())
    assert float(d[:, 0].mean()) <= 1e-5, float(d[:, 0].mean())
    assert float((out[False].proba_sel - out[True].proba_sel).abs().max()) <= 2e-4


def test_fused_logreg_guards_raise_after_launch(dev):
    """The fused device path reads its input guards (finite X, 0/1 labels) with the cooperative
    launch's error word in one transfer: bad inputs still raise, as the synchronous checks did."""
    from hfens.utils.guards import NonFiniteError
    from hfens.models import logreg_solver
    X = torch.randn(4000, 5, dtype=torch.float64, device=dev)
    y = (torch.arange(4000, device=dev) % 2).to(torch.float64)
    m = LogisticRegression().fit(X, y)
    assert logreg_solver.LAST_PATH["path"] == "fused"
    assert torch.isfinite(m.coef_).all()
    Xbad = X.clone()
    Xbad[17, 3] = float("nan")
    with pytest.raises(NonFiniteError):
        LogisticRegression().fit(Xbad, y)
    with pytest.raises(ValueError):
        LogisticRegression().fit(X, y * 2)


@pytest.mark.parametrize("rows,subsample,mf", [(70000, 1.0, "1"), (130000, 0.7, "1"), (70000, 1.0, "0")])
def test_gbdt_stage_persistent_bit_identical(dev, monkeypatch, rows, subsample, mf):
    """The persistent stage loop (ONE gbdt_stump_stage launch for every boosting stage, a device
    grid barrier between stages) gives the launch-per-stage loop's model bit for bit — trees,
    thresholds, leaf values, impurities, train_score_ — with sklearn's tie ranks, bagging and both
    histogram paths."""
    from hfens.models import hist_gbdt
    monkeypatch.setattr(hist_gbdt, "STUMP_PATH", "stage")
    monkeypatch.setattr(hist_gbdt, "FUSED_STUMPS", False)
    monkeypatch.setenv("HFENS_GBDT_MFMA", mf)
    X, y = _data(rows, 24, 67)
    g = torch.Generator().manual_seed(9)
    X[:, 3] = torch.randint(0, 2, (rows,), generator=g).double()
    X[:, 6] = torch.randint(0, 5, (rows,), generator=g).double()
    masks = torch.ones(3, rows, dtype=torch.bool)
    masks[1, ::5] = False
    masks[2, 2::5] = False
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(hist_gbdt, "PERSIST", mode)
        ms = [GradientBoostingClassifier(n_estimators=50, max_depth=1, subsample=subsample, random_state=s)
              for s in (2020, 7, 8)]
        fit_gbdt_batch(ms, X.to(dev), y.to(dev), masks.to(dev))
        assert hist_gbdt.LAST_PATH["path"] == "stage"
        assert hist_gbdt.GRAPH_INFO["persist"] == (mode == "1")
        out[mode] = _gbdt_outputs(ms)
    for a, b in zip(out["0"], out["1"]):
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_gbdt_persistent_barrier_timeout_falls_back(dev, monkeypatch):
    """A persistent-loop grid-barrier wait past its deadline (here injected at the first barrier:
    HFENS_GBDT_PERSIST_DEADLINE_MS < 0) no longer fails the fit: the boosting re-runs with one launch
    per stage in the same process and gives the launch-per-stage model bit for bit."""
    from hfens.models import hist_gbdt
    monkeypatch.setattr(hist_gbdt, "STUMP_PATH", "stage")
    monkeypatch.setattr(hist_gbdt, "FUSED_STUMPS", False)
    rows = 130000
    X, y = _data(rows, 24, 31)
    masks = torch.ones(2, rows, dtype=torch.bool)
    masks[1, ::3] = False
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(hist_gbdt, "PERSIST", mode)
        if mode == "1":
            monkeypatch.setenv("HFENS_GBDT_PERSIST_DEADLINE_MS", "-1")
            hist_gbdt.LAST_PATH.pop("persist_fallback", None)
        ms = [GradientBoostingClassifier(n_estimators=20, max_depth=1, random_state=s) for s in (3, 4)]
        if mode == "1":
            with pytest.warns(RuntimeWarning, match="deadline"):
                fit_gbdt_batch(ms, X.to(dev), y.to(dev), masks.to(dev))
            assert hist_gbdt.LAST_PATH.get("persist_fallback") == 1
            assert not hist_gbdt._PERSIST_OFF[0]
        else:
            fit_gbdt_batch(ms, X.to(dev), y.to(dev), masks.to(dev))
        out[mode] = _gbdt_outputs(ms)
    for a, b in zip(out["0"], out["1"]):
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_stump_ranks_device_matches_host(dev):
    """sklearn's root feature-visit order computed on the device (stackdev.hip gbdt_ranks_dev: each
    model's constant features from its rows' bins, the rand_r Fisher-Yates per tree) equals the host
    computation, including features constant on one model's rows only."""
    from hfens.models import hist_gbdt
    from hfens.models.binning import fit_bins
    X, _ = _data(4000, 17, 12)
    X[:, 4] = 1.0                                   # constant everywhere
    X[:, 6] = 0.0
    X[:5, 6] = 1.0                                  # constant on the rows of models that skip 0-4
    masks = torch.ones(4, 4000, dtype=torch.bool)
    masks[1, :5] = False
    masks[2, ::3] = False
    masks[3, 2000:] = False
    Xd = X.to(dev)
    bins = fit_bins(Xd, 256).transform(Xd).contiguous()
    ms = [GradientBoostingClassifier(n_estimators=60, max_depth=1, random_state=s) for s in (2020, 7, 2020, 8)]
    host = hist_gbdt.sklearn_stump_ranks(ms, bins, masks.to(dev), 60)
    devr = hist_gbdt.stump_ranks_device(ms, bins, masks.to(dev).float(), 60)
    assert torch.equal(host.cpu(), devr.cpu())


def test_stacking_device_bases_match_synchronous(dev, monkeypatch):
    """The host-synchronisation-free GBC / L1-LR fold batches (stack_trainer.DEVICE_BASES: deferred
    guards, device stump ranks, bins from the all-column map fitted under the LassoCV path, device
    out-of-fold columns) give the synchronous round-4 fit: the same refit trees and coefficients bit
    for bit, out-of-fold columns to the f32 tree-walk rounding of the old path (its forest kernel
    adds f32 leaf values; the device column is the f64 sum the reference's predict_proba forms)."""
    from hfens import pipeline
    from hfens.models import stack_trainer
    Xd, yd, names = make_hf_cohort(3000, 40, seed=93, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(1000, 40, seed=94, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(stack_trainer, "DEVICE_BASES", flag)
        monkeypatch.setattr(pipeline, "BIN_AHEAD", flag)   # (on: exercised here, off by default)
        out[flag] = pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev)
    m0, m1 = out[False].model, out[True].model
    assert np.array_equal(out[False].selected, out[True].selected)
    g0, g1 = m0.estimators_[1], m1.estimators_[1]
    for a in ("tree_feature_", "tree_threshold_", "tree_value_", "tree_impurity_", "train_score_"):
        assert torch.equal(getattr(g0, a).cpu(), getattr(g1, a).cpu()), a
    l0, l1 = m0.estimators_[2], m1.estimators_[2]
    assert torch.equal(l0.coef_.cpu(), l1.coef_.cpu()) and torch.equal(l0.intercept_.cpu(), l1.intercept_.cpu())
    d = (m0.oof_meta_ - m1.oof_meta_).abs()
    assert float(d[:, 0].max()) == 0.0                    # the SVC column is untouched
    assert float(d[:, 1].max()) <= 1e-6, float(d[:, 1].max())
    assert float(d[:, 2].max()) <= 1e-12, float(d[:, 2].max())
    assert float((out[False].proba_sel - out[True].proba_sel).abs().max()) <= 1e-5


def test_prelaunched_svc_batch_matches(dev, monkeypatch):
    """The SVC batch enqueued under the LassoCV path from the selector's DEVICE column list
    (stack_trainer.prelaunch_stack: device γ patched into the problem records, no host read before
    the SMO) fits the same stack as the batch launched after the host knows the selection: the same
    columns, γ to the last bits of a variance sum (device two-pass vs torch's), and the same model
    up to the f32 pair sequence that a last-bit γ change may alter."""
    from hfens import pipeline
    from hfens.models import stack_trainer
    Xd, yd, names = make_hf_cohort(6000, 40, seed=95, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(2000, 40, seed=96, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(stack_trainer, "PRELAUNCH_SVC", flag)
        out[flag] = pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev)
        assert stack_trainer.LAST_PRELAUNCH["used"] == flag
    assert np.array_equal(out[False].selected, out[True].selected)
    s0, s1 = out[False].model.estimators_[0].steps[1][1], out[True].model.estimators_[0].steps[1][1]
    assert abs(float(s0._gamma) - float(s1._gamma)) <= 1e-14 * float(s0._gamma)
    d = float((out[False].proba_sel - out[True].proba_sel).abs().max())
    assert d <= 2e-3, d
    assert abs(out[False].scores["auroc"] - out[True].scores["auroc"]) <= 2e-3


def test_lasso_speculation_hit_and_miss(dev, monkeypatch):
    """The speculative selection (lasso.SPECULATE: the smallest-alpha refit's columns, the SVC batch
    enqueued on them while the CV paths run).  Hit: the selection, α and model equal the
    non-speculative prelaunch (same device-γ batch on the same columns).  Forced miss (speculating on
    the LARGEST alpha): the batch is discarded and redone on the real selection, quietly, giving the
    non-prelaunched fit."""
    from hfens import pipeline
    from hfens.models import lasso, stack_trainer
    Xd, yd, names = make_hf_cohort(6000, 40, seed=95, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(2000, 40, seed=96, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]

    def run(spec, idx=-1, pre=True):
        monkeypatch.setattr(lasso, "SPECULATE", spec)
        monkeypatch.setattr(lasso, "SPEC_ALPHA_INDEX", idx)
        monkeypatch.setattr(stack_trainer, "PRELAUNCH_SVC", pre)
        stack_trainer.LAST_PRELAUNCH.clear()
        r = pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev)
        return r, dict(stack_trainer.LAST_PRELAUNCH)
    base, lp0 = run(False)
    hit, lp1 = run(True)
    assert lp0["used"] and lp1["used"] and lp1["speculative"] and not lp1.get("spec_miss")
    assert np.array_equal(base.selected, hit.selected)
    assert torch.equal(base.proba_sel, hit.proba_sel)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")        # a speculation miss is not a warning
        miss, lp2 = run(True, idx=0)
    assert lp2.get("spec_miss") == 1 and not lp2["used"]
    nopre, _ = run(False, pre=False)
    assert np.array_equal(miss.selected, nopre.selected)
    assert torch.equal(miss.proba_sel, nopre.proba_sel)


def test_prelaunched_svc_without_early_read(dev, monkeypatch):
    """the prelaunched (device-γ) SVC batch finished WITHOUT the early read-back
    (HFENS_SVC_EARLY_READ=0) reads the SMO error word itself and resolves γ — no UnboundLocalError —
    and fits the same stack as with the early read (the same solve; only the read-back differs)."""
    from hfens import pipeline
    from hfens.models import smo, stack_trainer
    Xd, yd, names = make_hf_cohort(6000, 40, seed=95, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(2000, 40, seed=96, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    out = {}
    for early in (True, False):
        monkeypatch.setattr(smo, "EARLY_READ", early)
        stack_trainer.LAST_PRELAUNCH.clear()
        out[early] = pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev)
        assert stack_trainer.LAST_PRELAUNCH["used"]
    assert np.array_equal(out[True].selected, out[False].selected)
    assert torch.equal(out[True].proba_sel, out[False].proba_sel)


def _task_worker(rank, world, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HFENS_DIST_REQUIRE_DEVICE="1")
    import torch.distributed as dist
    from hfens import pipeline
    from hfens.io.synth import make_hf_cohort
    from hfens.models import stack_trainer
    from hfens.parallel import dist as pdist
    from hfens.parallel.dist import all_gather_rows, shard_rows
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pdist.require_device_tensors()
    try:
        dev = torch.device("cuda:0")
        pipeline.DP_POLICY = "task"
        Xd, yd, names = make_hf_cohort(6000, 40, seed=95, nan_frac=0.02)
        Xs, ys, _ = make_hf_cohort(2000, 40, seed=96, nan_frac=0.02)
        a = [torch.as_tensor(shard_rows(v, rank, world), device=dev) for v in (Xd, yd, Xs, ys)]
        r = pipeline.develop(a[0], a[1], a[2], a[3], names, device=dev, group=dist.group.WORLD)
        p = all_gather_rows(r.proba_sel.double()[:, None], dist.group.WORLD)[:, 0]
        if rank == 0:
            q.put((r.selected.copy(), p.cpu().numpy(), dict(stack_trainer.LAST_PRELAUNCH),
                   r.model.oof_meta_.cpu().numpy(), _stack_params(r.model)))
    finally:
        pdist.shutdown()


def _stack_params(m):
    """The fitted refit models' parameters (host arrays) of a stacking fit."""
    svc = m.estimators_[0].steps[1][1]
    return [svc._dual_coef_.cpu().numpy(), svc._intercept_.cpu().numpy(), svc.support_.cpu().numpy(),
            np.array([svc._probA.item(), svc._probB.item()]), m.estimators_[1].tree_value_.cpu().numpy(),
            m.estimators_[1].tree_feature_.cpu().numpy(), m.estimators_[2].coef_.cpu().numpy(),
            m.final_estimator_.coef_.cpu().numpy(), m.final_estimator_.intercept_.cpu().numpy()]


@pytest.mark.parametrize("world", [2, 3])
def test_develop_task_policy_prelaunched_matches_single(dev, world):
    """the task policy (every rank holds every row, the SMO problems spread over the
    ranks) runs the single-process critical path — the speculative selection, the stacking fit
    prelaunched under the LassoCV path (device γ, device out-of-fold columns, the meta model) with
    the task-parallel SMO's one all-reduce inside it.  2 and 3 processes on one card (gloo, device
    tensors only): the stack's out-of-fold matrix and the held-out probabilities equal the single
    process's bit for bit (the solutions travel as their f64 bit patterns), and so do the refit
    models' parameters; the held-out rows are scored per shard (other batch shapes of the f32
    inference kernels), so within 1e-5."""
    import socket
    import torch.multiprocessing as mp
    from hfens import pipeline
    from hfens.io.synth import make_hf_cohort
    from hfens.models import stack_trainer
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_task_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    sel, p, lp, oof, params = q.get(timeout=150)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert lp["used"] and lp["speculative"] and not lp.get("spec_miss")
    Xd, yd, names = make_hf_cohort(6000, 40, seed=95, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(2000, 40, seed=96, nan_frac=0.02)
    a = [torch.as_tensor(v, device=dev) for v in (Xd, yd, Xs, ys)]
    r = pipeline.develop(a[0], a[1], a[2], a[3], names, device=dev)
    assert stack_trainer.LAST_PRELAUNCH["used"]
    assert np.array_equal(sel, r.selected)
    assert np.array_equal(oof, r.model.oof_meta_.cpu().numpy())
    for a, b in zip(params, _stack_params(r.model)):
        assert np.array_equal(a, b)
    assert float(np.abs(p - r.proba_sel.double().cpu().numpy()).max()) <= 1e-5


def test_stacking_persistent_gbc_and_fallback(dev, monkeypatch):
    """HFENS_GBDT_PERSIST_STACK: the stacking fit's deferred GBC batch as ONE persistent launch gives
    the launch-per-stage stack bit for bit; a forced barrier-deadline miss is caught
    by the deferred read, re-runs the batch per stage and refits the meta model — the same stack
    (deadline −1: the failure injected at the first barrier)."""
    from hfens import pipeline
    from hfens.io.synth import make_hf_cohort
    from hfens.models import hist_gbdt
    Xd, yd, names = make_hf_cohort(6000, 40, seed=95, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(2000, 40, seed=96, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    out = {}
    for tag, persist, deadline in (("launch", False, None), ("persist", True, None), ("miss", True, "-1")):
        monkeypatch.setattr(hist_gbdt, "PERSIST_STACK", persist)
        if deadline is not None:
            monkeypatch.setenv("HFENS_GBDT_PERSIST_DEADLINE_MS", deadline)
        hist_gbdt.LAST_PATH.pop("persist_fallback", None)
        import warnings
        with warnings.catch_warnings(record=True):
            warnings.simplefilter("always")
            out[tag] = pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev)
        out[tag + "_persist"] = hist_gbdt.GRAPH_INFO.get("persist")
        out[tag + "_fb"] = hist_gbdt.LAST_PATH.get("persist_fallback", 0)
    assert out["persist_persist"] and not out["launch_persist"] and out["persist_fb"] == 0
    assert out["miss_fb"] >= 1
    for tag in ("persist", "miss"):
        assert torch.equal(out["launch"].model.oof_meta_, out[tag].model.oof_meta_)
        assert torch.equal(out["launch"].proba_sel, out[tag].proba_sel)


def test_headline_fit_leaves_no_device_memory_in_reference_cycles(dev):
    """VERDICT r5 #5 (step outliers): the SMO batch state used to sit in reference cycles (the
    working-set runs' closures ↔ their dicts, finish_svc_batch's deferred closure ↔ its batch dict):
    ≈ 77 MB of device buffers per fit stayed allocated until a full collection, so the caching
    allocator grew by new segments every few steps (profiles/r6_runs/r6o, r6q).  After a fit, the
    collector must find no CUDA tensor in unreachable cycles and allocated memory must not grow."""
    import gc
    from hfens import pipeline
    from hfens.io.synth import make_hf_cohort
    Xd, yd, names = make_hf_cohort(6000, 40, seed=95, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(2000, 40, seed=96, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    for _ in range(2):
        pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev, evaluate=False)
    torch.cuda.synchronize()
    gc.collect()
    a0 = torch.cuda.memory_allocated(dev)
    was = gc.isenabled()
    gc.disable()
    try:
        pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev, evaluate=False)
        torch.cuda.synchronize()
        a1 = torch.cuda.memory_allocated(dev)
        gc.set_debug(gc.DEBUG_SAVEALL)
        gc.collect()
        leaked = [o for o in gc.garbage if isinstance(o, torch.Tensor) and o.is_cuda]
    finally:
        gc.set_debug(0)
        gc.garbage.clear()
        if was:
            gc.enable()
    assert not leaked, f"{len(leaked)} CUDA tensors in reference cycles"
    assert a1 - a0 <= (1 << 20), a1 - a0


def test_merged_oof_decisions_bit_identical(dev, monkeypatch):
    """stack_trainer.MERGED_OOF_DEC: the SVC's out-of-fold decisions computed inside the batch's
    Platt decision launch give the separate launch's out-of-fold column bit for bit (same partials;
    the longer launch only adds all-zero split columns)."""
    from hfens import pipeline
    from hfens.io.synth import make_hf_cohort
    from hfens.models import smo, stack_trainer
    Xd, yd, names = make_hf_cohort(6000, 40, seed=95, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(2000, 40, seed=96, nan_frac=0.02)
    args = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    out = {}
    for merged in (False, True):
        monkeypatch.setattr(stack_trainer, "MERGED_OOF_DEC", merged)
        out[merged] = pipeline.develop(args[0], args[1], args[2], args[3], names, device=dev)
    assert torch.equal(out[False].model.oof_meta_, out[True].model.oof_meta_)
    assert torch.equal(out[False].proba_sel, out[True].proba_sel)

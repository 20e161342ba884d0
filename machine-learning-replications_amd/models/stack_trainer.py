"""StackingClassifier.fit as batched device work (reference ``train_ensemble_public.py:61``;
sklearn ``ensemble/_stacking.py`` semantics).

Fit plan for the reference stack (3 base models × (5 OOF folds + full refit)):

1. StratifiedKFold(5) test folds (sklearn assignment) → 6 training masks.
2. svc pipeline: 6 StandardScaler fits (masked column moments) → 6 scaled training
   matrices → ONE ``fit_svc_batch`` (36 SMO problems in one launch).
3. gbc: ONE ``fit_gbdt_batch`` over the 6 masks (shared binned matrix).
4. lg: ONE ``fit_logreg_batch`` over the 6 masks.
5. OOF ``predict_proba[:, 1]`` of the 5 fold models on their test rows → meta features
   (svc, gbc, lg order) → final LR(L2, balanced).

With a process group: rows are sharded; GBDT / LR / scaler moments reduce across
ranks, the 36 SVM problems are split across ranks (task parallel) and the OOF
meta-features all-gathered (:mod:`hfens.parallel.stack`).

On the GPU the SVC batch (36 SMO problems = 36 workgroups: a few dozen of the 256 CUs, for
most of the fit) runs on its own HIP stream while GBC and LR run on the default stream — the
idle CUs do that work concurrently.  The SVC batch is enqueued first
(``launch_svc_batch``: no host sync after the SMO launch) and collected after GBC/LR, all from
one host thread — under a process group the SVC all-gathers, the GBC/LR all-reduces and the
SVC broadcasts are therefore issued in the same order on every rank on one communicator.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..utils.timing import StageTimer
from .gbdt import GradientBoostingClassifier
from .hist_gbdt import fit_gbdt_batch
from .linear import LogisticRegression
from .logreg_solver import finish_logreg_batch, fit_logreg_batch, launch_logreg_batch
from .model_selection import fold_masks, stratified_kfold_test_folds
from .scaler import StandardScaler
from .smo import finish_svc_batch, fit_svc_batch, launch_svc_batch
from .stacking import Pipeline
from .svc import SVC

N_FOLDS = 5
_TRACE_HOST = os.environ.get("HFENS_TRACE_HOST", "0") == "1"
CONCURRENT_BASES = os.environ.get("HFENS_CONCURRENT_BASES", "1") != "0"
# the SVC's out-of-fold column computed on the device behind the SMO (smo.enqueue_svc_oof) instead
# of by the fold models' predict_proba after their host bookkeeping
DEVICE_SVC_OOF = os.environ.get("HFENS_DEVICE_SVC_OOF", "1") != "0"
# with the SVC's out-of-fold column computed on the device, the five fold SVCs are never used
# again (the stacking fit keeps only the refit models, like StackingClassifier's
# cross_val_predict): their set_fitted (support-vector extraction, ≈ 0.3 ms of host work each) is
# skipped.  0 = finish them anyway.
SKIP_FOLD_SVC = os.environ.get("HFENS_SKIP_FOLD_SVC", "1") != "0"
# GBC and L1-LR fold batches enqueued with no host synchronisation (single process, GPU): their
# input / leaf guards and the LR launch's error word are read once after the SVC (utils.guards.Deferred),
# their out-of-fold columns come from the device node tables / coefficients (ops/csrc/stackdev.hip),
# and only the refit models are finished.  0 = the synchronous per-batch fits of round 4.
DEVICE_BASES = os.environ.get("HFENS_DEVICE_BASES", "1") != "0"
# the meta model's launch enqueued before the SVC's results are read back (0: after them)
EARLY_META = os.environ.get("HFENS_EARLY_META", "1") != "0"
# ... with its set_fitted done at that launch (the fit's tail then only reads its error word / guards)
META_PRESET = os.environ.get("HFENS_META_PRESET", "1") != "0"
# the GBC / L1-LR guards resolved BEFORE the SVC's read-back when their staged copy has already
# landed (they finish milliseconds before the SMO): off the tail's host path
BASES_EARLY_RESOLVE = os.environ.get("HFENS_BASES_EARLY_RESOLVE", "1") != "0"


def _kind(est):
    if isinstance(est, Pipeline):
        if not (isinstance(est.steps[0][1], StandardScaler) and isinstance(est.steps[-1][1], SVC)
                and len(est.steps) == 2):
            raise NotImplementedError("pipeline must be StandardScaler → SVC")
        return "svc"
    if isinstance(est, SVC):
        return "svc_raw"
    if isinstance(est, GradientBoostingClassifier):
        return "gbc"
    if isinstance(est, LogisticRegression):
        return "lr"
    raise NotImplementedError(f"unsupported base estimator {type(est).__name__}")


def _global_scaler_moments(X, masks, group):
    """Per-mask column mean / population variance over the rows of EVERY rank (two-pass, f64):
    one all-reduce of [count | Σx] per mask, then one of Σ(x − mean)² — 2 collectives for all
    masks.  A rank-local fit would scale each shard differently."""
    from ..parallel import dist as pdist
    Xd = X.to(torch.float64)
    m = masks.to(torch.float64)                                   # [K, n]
    cnt, s1 = pdist.all_reduce_sum_f64([m.sum(1), m @ Xd], group)
    mean = s1 / cnt[:, None]
    sq = torch.stack([(m[k][:, None] * (Xd - mean[k]) ** 2).sum(0) for k in range(m.shape[0])])
    (sq,) = pdist.all_reduce_sum_f64([sq], group)
    return mean, sq / cnt[:, None], cnt


def scaler_batch_device(X: torch.Tensor, rows_host):
    """The K fold scalers of the SVC pipeline in ONE native pass (ops/csrc/scaler.hip, SURVEY.md
    K2): per-subset mean / population variance (two-pass f64, deterministic) and every subset's
    scaled rows in one concatenated matrix.  Returns (means [K, F], vars [K, F], Z [Σ l, F],
    offsets, device row index)."""
    from .. import ops
    K = len(rows_host)
    lens = [int(r.shape[0]) for r in rows_host]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n, F = X.shape
    dev = X.device
    idx = _index_to(np.concatenate(rows_host).astype(np.int64), dev)
    offs_d = _index_to(offs, dev)
    max_rows = max(lens)
    S = min(64, max(1, -(-max_rows // 1024)))
    part = torch.empty(2 * K * S * 64, dtype=torch.float64, device=dev)
    mean = torch.empty(K, F, dtype=torch.float64, device=dev)
    var = torch.empty(K, F, dtype=torch.float64, device=dev)
    Z = torch.empty(int(offs[-1]), F, dtype=torch.float64, device=dev)
    Xc = X.to(torch.float64).contiguous()
    ops.ext().scaler_batch(Xc.data_ptr(), n, F, idx.data_ptr(), offs_d.data_ptr(), K, max_rows, part.data_ptr(),
                           mean.data_ptr(), var.data_ptr(), Z.data_ptr(), ops.stream_ptr(dev))
    return mean, var, Z, offs, idx


NATIVE_SCALER = os.environ.get("HFENS_NATIVE_SCALER", "1") != "0"


def _svc_inputs(est, X, y, masks, group=None, rows_host=None):
    """Clones, their SVC objects and the scaled per-mask training matrices.  ``group`` (rows
    sharded): the scalers are fitted on the global masked rows, as a single process would.
    ``rows_host``: the masks' row indices, known on the host (no ``nonzero`` synchronisation);
    on the GPU the fold scalers then run as one native batched fit + transform."""
    kind = _kind(est)
    clones = [est.clone() for _ in range(masks.shape[0])]
    Zs, ys = [], []
    if (kind == "svc" and group is None and rows_host is not None and X.is_cuda and NATIVE_SCALER
            and X.shape[1] <= 64):
        from .. import ops
        if ops.has_ext():
            mean, var, Z, offs, idx = scaler_batch_device(X, rows_host)
            ycat = y.index_select(0, idx)
            # every clone's scaler attributes from ONE sqrt / where over [K, F] (StandardScaler._set's
            # expressions, elementwise: the same bits as K separate calls)
            sd = torch.sqrt(var)
            scale = torch.where(sd == 0.0, torch.ones_like(sd), sd)
            for k, c in enumerate(clones):
                c.steps[0][1]._set_parts(mean[k], var[k], scale[k], int(offs[k + 1] - offs[k]))
                Zs.append(Z[offs[k]:offs[k + 1]])
                ys.append(ycat[offs[k]:offs[k + 1]])
            return clones, [c.steps[-1][1] for c in clones], Zs, ys
    gm = _global_scaler_moments(X, masks, group) if (group is not None and kind == "svc") else None
    for k, (c, m) in enumerate(zip(clones, masks)):
        rows = _index_to(rows_host[k], X.device) if rows_host is not None else torch.nonzero(m).squeeze(1)
        Xm = X[rows]
        if kind == "svc":
            sc = c.steps[0][1]
            if gm is None:
                sc.fit(Xm)
            else:
                sc._set(gm[0][k], gm[1][k], int(gm[2][k]))
            Zs.append(sc.transform(Xm))
        else:
            Zs.append(Xm)
        ys.append(y[rows])
    svcs = [c.steps[-1][1] if kind == "svc" else c for c in clones]
    return clones, svcs, Zs, ys


def fit_base_batch(est, X, y, masks, group=None, timer=None, svc_group=None, rows_host=None):
    """Fit ``masks.shape[0]`` clones of ``est`` on the masked row subsets; returns them.
    ``group``: rows sharded over ranks (data parallel); ``svc_group``: rows replicated on every
    rank, only the SMO problems are spread over the ranks (task parallel)."""
    kind = _kind(est)
    if kind in ("svc", "svc_raw"):
        clones, svcs, Zs, ys = _svc_inputs(est, X, y, masks, group, rows_host)
        if group is None:
            fit_svc_batch(svcs, Zs, ys, group=svc_group)
        else:
            from ..parallel.stack import fit_svc_batch_distributed
            fit_svc_batch_distributed(svcs, Zs, ys, group)
    elif kind == "gbc":
        clones = [est.clone() for _ in range(masks.shape[0])]
        fit_gbdt_batch(clones, X, y, masks, group=group)
    else:
        clones = [est.clone() for _ in range(masks.shape[0])]
        # masks are [fold 0 … fold K−1, refit]; scikit-learn fits the refit first (its seed draw
        # from the global RNG comes first, the liblinear emulation's draw order)
        nb = masks.shape[0]
        fit_logreg_batch(clones, X, y, masks, group=group, seed_order=[nb - 1] + list(range(nb - 1)))
    return clones


def _index_to(a, device) -> torch.Tensor:
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64))
    if torch.device(device).type != "cuda":
        return t
    return t.pin_memory().to(device, non_blocking=True)


def plan_stacking(clf, y_np: np.ndarray) -> dict:
    """The label-only bookkeeping of :func:`fit_stacking` — StratifiedKFold test folds, the fold row
    sets and every SVC fit's libsvm problem expansion with its Platt column maps — computed from the
    development labels alone, so the caller can run it on the host while earlier device work (the
    LassoCV path) is in flight, off the SVC launch's critical path."""
    from .smo import plan_svc_problems
    y_np = np.asarray(y_np, dtype=np.float64).reshape(-1)
    folds_np = stratified_kfold_test_folds(y_np, N_FOLDS)
    n = y_np.shape[0]
    rows_host = [np.nonzero(folds_np != k)[0] for k in range(N_FOLDS)] + [np.arange(n)]
    svc_pre = {}
    for i, (_, est) in enumerate(clf.estimators):
        if _kind(est) == "svc":
            pre = plan_svc_problems(est.steps[-1][1], [y_np[r] for r in rows_host])
            if pre is not None:
                svc_pre[i] = pre
    return dict(y_np=y_np, folds_np=folds_np, rows_host=rows_host, svc_pre=svc_pre)


NATIVE_PLAN = os.environ.get("HFENS_NATIVE_PLAN", "1") != "0"


def plan_stacking_start(clf, y_np: np.ndarray):
    """Start :func:`plan_stacking`'s label work on a helper thread in ONE native call with the GIL
    released (ops/csrc/host.hip stack_plan_host: folds + every fit's libsvm expansion), so it runs
    while the calling thread launches the imputation and the LassoCV prelude.  Returns ``join()`` →
    the plan (equal to plan_stacking's, array for array: tests/test_smo_host.py), or None when not
    eligible (no extension, labels not 0/1 of both classes, not one probability SVC pipeline)."""
    from .. import ops
    from . import smo
    y_np = np.ascontiguousarray(np.asarray(y_np, dtype=np.float64).reshape(-1))
    n = int(y_np.shape[0])
    svc_cols = [i for i, (_, e) in enumerate(clf.estimators) if _kind(e) == "svc"]
    if not (NATIVE_PLAN and ops.has_ext() and len(svc_cols) == 1 and n >= N_FOLDS):
        return None
    svc = clf.estimators[svc_cols[0]][1].steps[-1][1]
    if not svc.probability or not ((y_np == 0.0) | (y_np == 1.0)).all():
        return None
    c1 = int(np.count_nonzero(y_np))
    if min(c1, n - c1) < N_FOLDS:
        return None
    if smo.SOLVER == "exact" or (smo.SOLVER == "auto" and n < smo.WS_MIN_POINTS):
        return None      # (the stored-Gram solver's Platt column maps: plan_stacking)
    seed = smo.sklearn_libsvm_seed(svc.random_state) & 0xFFFFFFFF
    nf1 = N_FOLDS + 1
    folds = np.empty(n, dtype=np.int64)
    rows = np.empty(nf1 * n, dtype=np.int64)
    lens = np.empty(nf1, dtype=np.int64)
    out = np.empty(nf1 * 7 * n, dtype=np.int64)
    meta = np.empty(nf1 * 21, dtype=np.int64)
    E = ops.ext()
    done = _plan_worker().submit(E.stack_plan_host, y_np.ctypes.data, n, N_FOLDS, seed, folds.ctypes.data,
                                 rows.ctypes.data, lens.ctypes.data, out.ctypes.data, meta.ctypes.data)
    balanced = svc.class_weight == "balanced"

    def join():
        done.wait()
        if done.error is not None:
            raise done.error
        rows_host = [rows[f * n:f * n + int(lens[f])] for f in range(nf1)]
        pre = []
        for f in range(nf1):
            l = int(lens[f])
            yf = y_np[rows_host[f]]
            mf = meta[f * 21:(f + 1) * 21]
            # 'balanced': l / (2·[#class 0, #class 1]) from the expansion's class-0 count (= the
            # bincount of _class_weights_host, the same f64 expression)
            cw = (l / (2 * np.array([mf[0], l - mf[0]], dtype=np.float64)) if balanced
                  else smo._class_weights_host(svc, yf))
            probs, mt = smo._wrap_expansion(f, l, out[f * 7 * n:(f + 1) * 7 * n], mf, None, cw, svc)
            pre.append((yf, probs, mt))
        return dict(y_np=y_np, folds_np=folds, rows_host=rows_host, svc_pre={svc_cols[0]: pre})
    return join


class _Done:
    """Completion of one :class:`_PlanWorker` job."""

    def __init__(self):
        import threading
        self._ev = threading.Event()
        self.error = None

    def wait(self):
        self._ev.wait()


class _PlanWorker:
    """One long-lived daemon thread running native host jobs (GIL released inside them) — a thread
    start per fit cost ≈ 0.1 ms of the launching thread's time (scripts/probes/preparts_profile.py)."""

    def __init__(self):
        import queue
        import threading
        self._q = queue.SimpleQueue()
        self._th = threading.Thread(target=self._run, name="hfens-plan-native", daemon=True)
        self._th.start()

    def _run(self):
        while True:
            fn, args, done = self._q.get()
            try:
                fn(*args)
            except BaseException as e:   # re-raised by the joining thread
                done.error = e
            done._ev.set()

    def submit(self, fn, *args) -> _Done:
        done = _Done()
        self._q.put((fn, args, done))
        return done


_PLAN_WORKER: list = []


def _plan_worker() -> _PlanWorker:
    if not _PLAN_WORKER:
        _PLAN_WORKER.append(_PlanWorker())
    return _PLAN_WORKER[0]


def _launch_svc(stc) -> bool:
    """SVC batch on a side stream ∥ the other base models on a second stream (:func:`_launch_bases`),
    from one host thread: everything ENQUEUED, nothing read back (:func:`_finish_concurrent`
    completes it).  Returns False when not applicable (the caller then fits sequentially)."""
    clf, X, y, masks, group = stc["clf"], stc["X"], stc["y"], stc["masks"], stc["group"]
    svc_group, rows_host, y_np, svc_pre = stc["svc_group"], stc["rows_host"], stc["y_np"], stc["svc_pre"]
    oof, early, dev_bases = stc["oof"], stc["early"], stc["dev_bases"]
    kinds = [_kind(e) for _, e in clf.estimators]
    svc_cols = [i for i, k in enumerate(kinds) if k in ("svc", "svc_raw")]
    if not (X.is_cuda and CONCURRENT_BASES and svc_cols and len(kinds) > len(svc_cols)):
        return False
    dev = X.device
    if group is not None:
        from ..parallel.stack import launch_svc_batch_distributed
    # two pool streams (the legacy default stream would implicitly serialise with them); the SVC
    # stream at high priority: HIP multiplexes streams onto GPU_MAX_HW_QUEUES hardware queues and
    # two same-priority pool streams were measured landing on ONE queue (serialised)
    # process-lifetime streams: fresh pool streams per fit defeat the caching allocator's
    # per-stream block reuse (hfens/runtime.py)
    from .. import runtime
    main = torch.cuda.current_stream(dev)
    side, other = runtime.stream(dev, "svc", priority=-1), runtime.stream(dev, "bases")
    side.wait_stream(main)
    if stc.get("x_event") is not None:
        # (the prelaunch: X is produced on the SVC stream from the speculative selection)
        side.wait_event(stc["x_event"])
    out, pending = {}, {}
    from ..utils.timing import hmark, dmark
    hmark("fit_bases")
    # every collective is issued from this thread in the same order on every rank:
    # SVC all-gathers / the task-parallel SMO all-reduce → GBC/LR all-reduces → SVC broadcasts
    with torch.cuda.stream(side):
        for i in svc_cols:
            clones, svcs, Zs, ys = _svc_inputs(clf.estimators[i][1], X, y, masks, group, rows_host)
            hmark("svc_inputs")
            if group is None:
                plan_i = (svc_pre or {}).get(i)
                yh = ([y_np[r] for r in rows_host] if (plan_i is None and y_np is not None and rows_host is not None)
                      else None)
                # the out-of-fold rows, scaled by their fold's scaler, go into the SVC batch's Platt
                # decision launch (one launch for both) — built when the batch asks for them (its
                # post-SMO tables, after the cascade parts and the first rounds are enqueued)
                memo = {}

                def items_of(clones=clones, memo=memo):
                    if "v" not in memo:
                        memo["v"] = stc["oof_items"](clones)
                    return memo["v"]
                merged = (stc["oof_svc_dev"] is not None and MERGED_OOF_DEC and stc["oof_items_ok"](clones))
                # device γ (no host read before the SMO) whenever the batch is eligible
                st = launch_svc_batch(svcs, Zs, ys, group=svc_group, y_host=yh, plan=plan_i,
                                      gamma_dev=GAMMA_DEV,
                                      oof_items=(lambda: [(k, Zt) for k, Zt, _ in items_of()]) if merged else None)
                items = items_of() if stc["oof_svc_dev"] is not None else None
                if stc["oof_svc_dev"] is not None:
                    # the OOF column straight from the device solution, behind the SMO on this
                    # stream: no wait for the fitted models' host bookkeeping
                    st["oof_dev"] = stc["oof_svc_dev"](i, clones, st, items)
                pending[i] = (clones, st)
            else:
                pending[i] = (clones, launch_svc_batch_distributed(svcs, Zs, ys, group))
            hmark("svc_launched")
    stc.update(pending=pending, out=out, side=side, other=other, main=main, svc_cols=svc_cols, bases_done=False)
    return True


def _launch_bases(stc):
    """The GBC / L1-LR fold batches on the "bases" stream (device out-of-fold columns), then the
    meta model's early launch behind every out-of-fold column."""
    clf, X, y, masks, group = stc["clf"], stc["X"], stc["y"], stc["masks"], stc["group"]
    oof, early, dev_bases = stc["oof"], stc["early"], stc["dev_bases"]
    side, other, main, svc_cols, out, pending = (stc["side"], stc["other"], stc["main"], stc["svc_cols"],
                                                 stc["out"], stc["pending"])
    from ..utils.timing import hmark, dmark
    other.wait_stream(main)
    if stc.get("x_event") is not None:
        other.wait_event(stc["x_event"])
        X.record_stream(other)
    # cooperative LR members must all fit on the CUs a cooperative SMO leaves free
    from . import logreg_solver, smo as _smo
    lr_budget = logreg_solver.BLOCK_BUDGET[0]
    if _smo.LAST_SMO_INFO.get("solver") in ("coop", "coop-otf"):
        logreg_solver.BLOCK_BUDGET[0] = max(1, _smo.COOP_RESERVE_CUS // 2)
    elif _smo.LAST_SMO_INFO.get("solver") == "ws" and X.is_cuda:
        # the working-set solver holds one CU per problem (its gradient updates come and go)
        logreg_solver.BLOCK_BUDGET[0] = max(1, _smo._num_cus(X.device) - int(_smo.LAST_SMO_INFO["problems"]) - 8)
    try:
        with torch.cuda.stream(other):
            # the L1-LR batch (one ≈ 2 ms cooperative launch) before the GBC's 100-stage loop: the
            # meta model waits for both, and the LR behind the GBC ended last (r6i: lg_done 17.9 vs
            # the SVC's out-of-fold column at 17.5 ms)
            order = [i for i in range(len(clf.estimators)) if i not in svc_cols]
            if LR_FIRST and dev_bases is not None:
                for i in order:
                    if _kind(clf.estimators[i][1]) == "gbc":
                        dev_bases["prebin"](clf.estimators[i][1])
                        hmark("gbc_prebinned")
                        break
                order.sort(key=lambda i: 0 if _kind(clf.estimators[i][1]) == "lr" else 1)
            for i in order:
                name, est = clf.estimators[i]
                r = dev_bases["fit"](i, est) if dev_bases is not None else None
                if r is not None:
                    out[i] = r        # enqueued, out-of-fold column on the device
                else:
                    out[i] = fit_base_batch(est, X, y, masks, group=group)
                    if oof is not None:
                        oof(i, out[i])
                hmark(f"{name}_host_done")
                dmark(f"{name}_done")
            # every meta-feature column of these bases is enqueued on this stream by now: the
            # meta model waits for this point, not for the bookkeeping enqueued after it
            cols_ev = torch.cuda.Event()
            cols_ev.record(other)
            if dev_bases is not None:
                # the refit models' fitted state from the device node tables / coefficients,
                # enqueued on this stream behind their solves while the SMO runs (no host read:
                # the guards are read after it)
                for f in dev_bases["post"]:
                    f()
                dev_bases["deferred"].stage()   # (their guards' read-back, queued right here)
                hmark("bases_post")
    finally:
        logreg_solver.BLOCK_BUDGET[0] = lr_budget
    if early is not None and pending and all(st.get("oof_dev") for _, st in pending.values()):
        # every meta-feature column is enqueued on the device: the meta model's launch goes in
        # now, before the SVC's results are read back — on the SVC stream, behind the SVC's own
        # out-of-fold kernel.  (On the main stream its wait for the SVC would be the head of an
        # otherwise idle hardware queue for the rest of the SMO: measured, such a pending
        # cross-stream wait slowed the SMO's dispatches by 2-4 ms, profiles/r5_headline.md.)
        hmark("early_in")
        side.wait_stream(main)
        side.wait_event(cols_ev)
        with torch.cuda.stream(side):
            early["handle"] = early["launch"]()
    stc["bases_done"] = True


def _finish_concurrent(stc):
    """Read back and complete what :func:`_launch_concurrent` enqueued; returns the fitted clone
    lists in estimator order."""
    from ..utils.timing import hmark, hmarks_flush
    group, pending, out, early, oof = stc["group"], stc["pending"], stc["out"], stc["early"], stc["oof"]
    side, other, main, dev_bases = stc["side"], stc["other"], stc["main"], stc["dev_bases"]
    if group is not None:
        from ..parallel.stack import finish_svc_batch_distributed
    with stc["timer"].stage("fit_bases(svc || gbc+lr)"):
        resolved = False
        if dev_bases is not None and BASES_EARLY_RESOLVE and dev_bases["deferred"].ready():
            # (their kernels have finished: the read is a look at host memory.  A fallback hook
            # re-solves on the caller's stream, after the bases' own)
            main.wait_stream(other)
            dev_bases["deferred"].resolve()
            resolved = True
            hmark("bases_resolved_early")
        # (the refit SVC's bookkeeping stays on the SVC stream: on the caller's stream its wait
        # for the SMO, pending at the head of an idle queue, slowed the SMO itself — 22.7 vs 19.3
        # ms / fit; on a new stream the stream → hardware-queue mapping moved and the GBC / LR
        # stream shared a queue with an SMO group — 20.4 ms)
        with torch.cuda.stream(side):
            for i, (clones, st) in pending.items():
                if group is None:
                    # with the out-of-fold column already on the device only the refit model is
                    # needed (finish_svc_batch leaves the fold models to st["finish_rest"])
                    dev_oof = bool(st.get("oof_dev")) and SKIP_FOLD_SVC
                    finish_svc_batch(st, defer=set(range(N_FOLDS)) if dev_oof else None)
                else:
                    finish_svc_batch_distributed(st, group)
                out[i] = clones
                if st.get("resolved") and early is not None:
                    early["stale"] = True      # (re-solved: the device OOF it was launched on is stale)
                if oof is not None and not (st.get("oof_dev") and not st.get("resolved")):
                    oof(i, clones)
        hmark("svc_finished")
        main.wait_stream(side)
        main.wait_stream(other)
        if dev_bases is not None and not resolved:
            # the GBC / LR guards and error words: ONE read, long after their kernels finished
            dev_bases["deferred"].resolve()
            hmark("bases_resolved")
    hmarks_flush()
    return [out[i] for i in range(len(stc["clf"].estimators))]


PRELAUNCH_SVC = os.environ.get("HFENS_PRELAUNCH_SVC", "1") != "0"
# the prelaunch enqueues the WHOLE stacking fit (GBC / L1-LR fold batches and the meta model too, not
# only the SVC batch) on the speculative selection: the bases' chain (≈ 7 ms from the selection) ran
# after lasso_fit before and ended beside the SMO (profiles/r6_runs/r6a: lg_done 18.1 vs svc_oof 18.5 ms).
# The bases go in right behind the SVC batch (prelaunch_bases from the early overlap; after the CV
# paths with pipeline.BASES_AFTER_CV — measured slower, profiles/r6_runs/r6e)
PRELAUNCH_BASES = os.environ.get("HFENS_PRELAUNCH_BASES", "1") != "0"
# device γ for the stacking fit's SVC batch whenever eligible (working-set solver, planned labels,
# gamma='scale'): no host read of the scaled rows' variance before the SMO, prelaunched or not
GAMMA_DEV = os.environ.get("HFENS_SVC_GAMMA_DEV", "1") != "0"
# the GBC / LR / meta device state (index uploads, label prep) built before the SVC batch is enqueued
# ("before") or after it on the bases stream ("after", default: the SVC batch's host enqueue starts
# ≈ 0.4 ms earlier; same fit time on one box, 18.99 / 18.19 vs 19.03 / 18.23 ms, profiles/r6_runs/r6i);
# built after it on the CALLER's stream it made the GBC's host bin fit wait for the whole SMO
# (profiles/r6_runs/r6h: gbc_binned 16.7 ms)
BASES_SETUP = os.environ.get("HFENS_BASES_SETUP", "after")
LR_FIRST = os.environ.get("HFENS_LR_FIRST", "1") != "0"
# the SVC's out-of-fold decisions computed in the batch's Platt decision launch (one launch, the same
# partials bit for bit: extra all-zero split columns add exact zeros)
MERGED_OOF_DEC = os.environ.get("HFENS_MERGED_OOF_DEC", "1") != "0"
LAST_PRELAUNCH = {"used": False}


def prelaunch_stack(clf, X_full: torch.Tensor, cols_dev: torch.Tensor, y: torch.Tensor, plan: dict,
                    svc_group=None):
    """Enqueue the stacking fit (scaler fits, the 36 SMO problems, Platt, the device out-of-fold
    columns, the GBC / L1-LR fold batches and the meta model) BEFORE the selected columns are known
    on the host: ``cols_dev`` is SelectFromModel's device column list, ``X_full`` the imputed
    development rows.  Everything else is label-only (``plan``: plan_stacking), γ is computed on the
    device (smo.launch_svc_batch gamma_dev), so nothing here waits for the selection — pipeline.develop
    calls it under the LassoCV path and the fit starts as soon as the (speculative) selection exists.
    ``svc_group``: the task-parallel policy (every rank holds every row; only the SMO problems are
    spread over the ranks).  Returns the state :func:`fit_stacking` finishes (after checking the host's
    selection against ``cols_dev``), or None when the stack is not eligible."""
    kinds = [_kind(e) for _, e in clf.estimators]
    svc_cols = [i for i, k in enumerate(kinds) if k == "svc"]
    if not (PRELAUNCH_SVC and X_full.is_cuda and CONCURRENT_BASES and DEVICE_SVC_OOF and svc_cols
            and len(kinds) > len(svc_cols) and plan.get("svc_pre") and all(i in plan["svc_pre"] for i in svc_cols)):
        return None
    from .. import runtime
    from .smo import use_lowrank
    dev = X_full.device
    n = int(X_full.shape[0])
    y_np, rows_host = plan["y_np"], plan["rows_host"]
    if int(y_np.shape[0]) != n:
        return None
    if use_lowrank([len(r) for r in rows_host], int(cols_dev.shape[0]), "cuda"):
        # the Nyström interior point is driven from the host (a synchronisation per iteration):
        # launched here it would hold this thread for the whole solve instead of running beside
        # the GBC / LR fits, as it does from the stacking trainer's streams
        return None
    from ..utils.timing import hmark
    hmark("pre_masks")
    main = torch.cuda.current_stream(dev)
    side = runtime.stream(dev, "svc", priority=-1)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        X = X_full.index_select(1, cols_dev)
        x_ev = torch.cuda.Event()
        x_ev.record(side)
    for t in (X_full, cols_dev, y):
        t.record_stream(side)
    stc = launch_stacking(clf, X, y, group=None, svc_group=svc_group, plan=plan, x_event=x_ev, bases=False)
    hmark("svc_prelaunched")
    return dict(cols_dev=cols_dev, X=X, state=stc)


def prelaunch_bases(pre) -> None:
    """The GBC / L1-LR batches and the meta model of a :func:`prelaunch_stack` state, enqueued (the
    pipeline calls it under the LassoCV path right after the CV paths are launched: the SVC batch
    first, the LassoCV's own paths second, the bases last — each waits on the host before it)."""
    stc = pre["state"] if pre is not None else None
    if stc is not None and PRELAUNCH_BASES and stc["concurrent"] and not stc["bases_done"]:
        _launch_bases(stc)


def launch_stacking(clf, X: torch.Tensor, y: torch.Tensor, timer: StageTimer = None, group=None, svc_group=None,
                    plan=None, x_event=None, bases: bool = True) -> dict:
    """The enqueue half of :func:`fit_stacking`: folds, masks, the SVC batch, the GBC / LR batches
    (``bases``; otherwise they are fitted in :func:`finish_stacking`) and the meta model's launch,
    with no host read on the single-process GPU path.  ``x_event``: X is produced on the SVC stream
    (the prelaunch); the streams wait for it."""
    timer = timer or StageTimer(enabled=False)
    from ..utils.timing import hmark as _hmk
    _hmk("stack_in")
    dev = X.device
    n = X.shape[0]
    y_np = None
    svc_pre = None
    if plan is not None and group is None and plan.get("y_np") is not None and int(plan["y_np"].shape[0]) == n:
        # folds, row sets and SVC problem expansions computed ahead from the same labels (plan_stacking)
        y_np, folds_np, svc_pre = plan["y_np"], plan["folds_np"], plan["svc_pre"]
    elif group is None:
        y_np = y.cpu().numpy().astype(np.float64)
        folds_np = stratified_kfold_test_folds(y_np, N_FOLDS)
    else:
        from ..parallel import dist as pdist
        folds_np = pdist.sharded_stratified_folds(y, N_FOLDS, group).cpu().numpy()
    rows_host = (plan["rows_host"] if svc_pre is not None
                 else [np.nonzero(folds_np != k)[0] for k in range(N_FOLDS)] + [np.arange(n)])
    masks = fold_masks(folds_np, N_FOLDS, device=dev)        # [6, n]
    # OOF rows per fold as device index tensors (ONE upload, non-blocking, split into per-fold views:
    # a stable argsort lists each fold's rows in ascending order, as np.nonzero does): the
    # meta-feature gathers / scatters then need no host synchronisation
    f8 = np.asarray(folds_np).astype(np.int8)      # (fold ids < 128: numpy's stable sort is a radix sort)
    order = np.argsort(f8, kind="stable")
    cnt = np.bincount(f8, minlength=N_FOLDS)
    order_d = _index_to(order, dev)
    starts = np.concatenate([[0], np.cumsum(cnt)])
    test_idx = [order_d[int(starts[k]):int(starts[k + 1])] for k in range(N_FOLDS)]
    meta = torch.zeros(n, len(clf.estimators), dtype=torch.float64, device=dev)
    stc = dict(clf=clf, X=X, y=y, masks=masks, test_idx=test_idx, meta=meta, group=group, svc_group=svc_group,
               rows_host=rows_host, y_np=y_np, svc_pre=svc_pre, folds_np=folds_np, timer=timer, plan=plan,
               x_event=x_event, concurrent=False)

    def oof(col, fitted):
        from ..utils.timing import hmark
        hmark(f"oof{col}")
        for k in range(N_FOLDS):
            if test_idx[k].numel():
                p1 = fitted[k].predict_proba(X.index_select(0, test_idx[k]))[:, 1].to(torch.float64)
                meta[:, col].index_copy_(0, test_idx[k], p1)

    def oof_items_ok(fitted):
        return DEVICE_SVC_OOF and all(hasattr(c, "steps") for c in fitted[:N_FOLDS])

    def oof_items(fitted):
        if not oof_items_ok(fitted):
            return None
        return [(k, fitted[k].steps[0][1].transform(X.index_select(0, test_idx[k])), test_idx[k])
                for k in range(N_FOLDS) if test_idx[k].numel()]

    def oof_svc_dev(col, fitted, st, items=None):
        items = items if items is not None else oof_items(fitted)
        if items is None:
            return False
        from .smo import enqueue_svc_oof
        return enqueue_svc_oof(st, items, meta, col)

    y64 = y.to(torch.float64)
    stc.update(oof=oof, oof_svc_dev=oof_svc_dev if group is None else None, oof_items=oof_items,
               oof_items_ok=oof_items_ok, y64=y64)
    _hmk("stack_prep")

    def new_final():
        return clf.final_estimator.clone() if clf.final_estimator is not None else LogisticRegression()
    stc["new_final"] = new_final
    stc.update(early=None, dev_bases=None)

    def bases_state():
        early = None
        if group is None and EARLY_META:
            fm = [new_final()]
            # the meta model's label-only inputs now, on this (otherwise idle) stream: behind the
            # out-of-fold columns only the features' guard and the intercept column remain
            from .logreg_solver import logreg_label_prep
            lprep = logreg_label_prep(fm, y64, n, dev) if X.is_cuda else None
            early = {"launch": lambda: launch_logreg_batch(fm, meta, y64, prep=lprep, preset=META_PRESET)}
        dev_bases = None
        if group is None and X.is_cuda and DEVICE_BASES:
            dev_bases = _device_bases(clf, X, y, masks, folds_np, meta, plan, early, oof)
        stc.update(early=early, dev_bases=dev_bases)
    if BASES_SETUP == "before" or not X.is_cuda:
        bases_state()
        stc["concurrent"] = _launch_svc(stc)
    else:
        # the SVC batch first (the fit's critical path); the other bases' device state after it, on
        # the bases stream
        stc["concurrent"] = _launch_svc(stc)
        from .. import runtime
        other = runtime.stream(dev, "bases")
        other.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(other):
            bases_state()
    if stc["concurrent"] and bases:
        _launch_bases(stc)
    return stc


def finish_stacking(stc):
    """Complete :func:`launch_stacking`: read the SVC / base models back, fit (or collect) the meta
    model and set the StackingClassifier's fitted attributes."""
    clf, timer, group, svc_group = stc["clf"], stc["timer"], stc["group"], stc["svc_group"]
    X, y, masks, meta, y64, early = stc["X"], stc["y"], stc["masks"], stc["meta"], stc["y64"], stc["early"]
    from ..utils.timing import hmark as _hmf
    _hmf("finish_in")
    if stc["concurrent"] and not stc["bases_done"]:
        _launch_bases(stc)        # (prelaunched without the bases: PRELAUNCH_BASES=0)
    fitted_all = _finish_concurrent(stc) if stc["concurrent"] else None
    full = []
    for col, (name, est) in enumerate(clf.estimators):
        if fitted_all is not None:
            fitted = fitted_all[col]        # OOF column already filled on the fitting stream
        else:
            with timer.stage(f"fit_{name}"):
                fitted = fit_base_batch(est, X, y, masks, group=group, svc_group=svc_group,
                                        rows_host=stc["rows_host"])
            with timer.stage(f"oof_{name}"):
                stc["oof"](col, fitted)
        full.append(fitted[N_FOLDS])
    with timer.stage("fit_meta"):
        from ..utils.timing import dmark, hmark as _hm
        _hm("meta_in")
        dmark("meta_in")
        if early is not None and "handle" in early and not early.get("stale"):
            final, = finish_logreg_batch(early["handle"])
        else:
            final = stc["new_final"]()
            fit_logreg_batch([final], meta, y64, group=group)
        dmark("meta")
    from ..utils.timing import hmark, hmarks_flush
    hmark("meta_done")
    clf.estimators_ = full
    clf.final_estimator_ = final
    clf.stack_method_ = ["predict_proba"] * len(full)
    clf.classes_ = torch.tensor([0.0, 1.0], dtype=torch.float64)
    clf.oof_meta_ = meta
    hmark("stack_done")
    hmarks_flush("[host-meta]")
    return clf


def _device_bases(clf, X, y, masks, folds_np, meta, plan, early, oof):
    """Host-synchronisation-free GBC / L1-LR fold batches for :func:`_fit_bases_concurrent`
    (:data:`DEVICE_BASES`).  ``fit(col, est)`` enqueues one estimator's 6 fits and its out-of-fold
    column (rows of fold k predicted by fold model k, written into ``meta[:, col]``), or returns None
    for estimators it does not handle; ``deferred`` / ``post`` complete them after the SVC."""
    from .. import ops
    from ..utils.guards import Deferred
    from .logreg_solver import launch_logreg_batch, set_fitted_from
    dev = X.device
    n, F = X.shape
    rows_np = np.concatenate([np.nonzero(folds_np == k)[0] for k in range(N_FOLDS)]).astype(np.int64)
    model_np = np.concatenate([np.full(int((folds_np == k).sum()), k, dtype=np.int32) for k in range(N_FOLDS)])
    oof_rows, oof_model = _index_to(rows_np, dev), _index_to(model_np, dev).to(torch.int32)
    m = int(rows_np.shape[0])
    Xc = X.to(torch.float64).contiguous()
    deferred, post, keep = Deferred(), [], []
    nb = int(masks.shape[0])
    E = ops.ext()

    box = {}

    def prebin(est):
        """The GBC's bin map (its host fit reads X back: done before anything else is queued on
        the bases stream, so that read does not wait for another base's solve)."""
        from .binning import fit_bins
        # (the inputs' guards are queued by the fit itself, on the deferred read)
        bm = fit_bins(Xc, int(est.max_bins))
        box["binned"] = (bm, bm.transform(Xc).contiguous())

    def gbc(col, est):
        clones = [est.clone() for _ in range(nb)]
        binned = box.pop("binned", None)
        ba, cols = (plan or {}).get("bins_all"), (plan or {}).get("cols")
        if binned is None and ba is not None and cols is not None and int(ba.max_bins) == int(clones[0].max_bins):
            bm = ba.select(cols)     # binned under the LassoCV path (pipeline.develop), columns selected here
            binned = (bm, bm.transform(Xc).contiguous())
        so = {}
        fit_gbdt_batch(clones, Xc, y, masks, binned=binned, deferred=deferred, finish={nb - 1}, state_out=so)
        st, raw0 = so["st"], so["raw0"].contiguous()

        def column(so_, st_, raw0_):
            E.oof_trees(Xc.data_ptr(), F, oof_rows.data_ptr(), oof_model.data_ptr(), m, so_["T"], nb, so_["NN"],
                        st_.feat.data_ptr(), st_.thr.data_ptr(), st_.value.data_ptr(), raw0_.data_ptr(), so_["lr"],
                        meta.data_ptr(), int(meta.shape[1]), col, ops.stream_ptr(dev))
        column(so, st, raw0)
        keep.append((st, raw0))
        post.append(so["finish"])
        if getattr(st, "persist_err", None) is not None:
            def on_fail(_v):
                # a barrier wait of the persistent stage loop passed its deadline: the trees are
                # partial — re-run the batch with one launch per stage (same trees, bit for bit), its
                # out-of-fold column, and the meta model launched on the stale one is refitted
                import warnings
                from . import hist_gbdt
                warnings.warn("GBDT persistent stage loop: a barrier wait passed its deadline; re-running "
                              "the stacking GBC batch with one launch per stage", RuntimeWarning)
                hist_gbdt.LAST_PATH["persist_fallback"] = hist_gbdt.LAST_PATH.get("persist_fallback", 0) + 1
                hist_gbdt._PERSIST_OFF[0] = True
                try:
                    so2 = {}
                    fit_gbdt_batch(clones, Xc, y, masks, binned=binned, finish={nb - 1}, state_out=so2)
                finally:
                    hist_gbdt._PERSIST_OFF[0] = False
                column(so2, so2["st"], so2["raw0"].contiguous())
                keep.append((so2["st"], so2["raw0"]))
                if early is not None:
                    early["stale"] = True
            deferred.word(st.persist_err, on_fail)
        return clones

    def lr(col, est):
        clones = [est.clone() for _ in range(nb)]
        # masks are [fold 0 … fold K−1, refit]; scikit-learn fits the refit first (seed draw order)
        h = launch_logreg_batch(clones, Xc, y, masks, seed_order=[nb - 1] + list(range(nb - 1)))
        if "fused" not in h:        # host emulation / loop path: fitted already
            if oof is not None:
                oof(col, clones)
            return clones
        fz = h["fused"]
        W, F1 = fz["args"][12], int(fz["args"][2])

        def column():
            E.oof_linear(Xc.data_ptr(), F, oof_rows.data_ptr(), oof_model.data_ptr(), m, W.data_ptr(), F1,
                         int(h["fit_intercept"]), float(h["scale"]), meta.data_ptr(), int(meta.shape[1]), col,
                         ops.stream_ptr(dev))
        column()
        if fz["flags"] is not None:
            deferred.flag(fz["flags"][0], "finite", "LogisticRegression.fit X")
            deferred.flag(fz["flags"][1], "binary", "LogisticRegression.fit y")
            fz["flags"] = None
        if fz["err"] is not None:
            def on_fail(_v):
                # a cooperative member timed out: the one-workgroup re-solve, a fresh column, and the
                # meta model launched on the stale one is refitted
                import warnings
                from . import logreg_solver
                warnings.warn("cooperative logistic regression timed out waiting for a member; re-solving "
                              "with one workgroup per model")
                logreg_solver.LAST_PATH["coop_fallback"] = True
                logreg_solver._launch_single(fz)
                column()
                set_fitted_from(h, only={nb - 1})     # (its intercept is a copy, not a view of W)
                if early is not None:
                    early["stale"] = True
            deferred.word(fz["err"], on_fail)
        post.append(lambda: set_fitted_from(h, only={nb - 1}))
        return clones

    def fit(col, est):
        kind = _kind(est)
        if kind == "gbc":
            return gbc(col, est)
        if kind == "lr":
            return lr(col, est)
        return None

    return dict(fit=fit, deferred=deferred, post=post, keep=keep, prebin=prebin)


def finish_prelaunched(pre: dict, timer: StageTimer = None) -> None:
    """Finish a :func:`prelaunch_stack` state before its selection is confirmed (pipeline.develop,
    while the LassoCV paths still run); :func:`fit_stacking` then only checks the selection — and
    refits from scratch on a miss."""
    stc = pre["state"]
    stc["timer"] = timer or stc["timer"]
    finish_stacking(stc)
    pre["finished"] = True


def fit_stacking(clf, X: torch.Tensor, y: torch.Tensor, timer: StageTimer = None, group=None, svc_group=None,
                 plan=None):
    pre = plan.get("prelaunch") if (plan is not None and group is None) else None
    from ..utils.timing import hmark
    hmark("stack_check_in")
    if pre is not None:
        # the stack was enqueued from the device column selection (prelaunch_stack): it is this
        # fit's only if the host's selection agrees (a speculation on the smallest alpha can miss)
        cols = plan.get("cols")
        LAST_PRELAUNCH["speculative"] = bool(pre.get("speculative"))
        ch = pre.get("cols_host")
        if ch is not None:
            from ..utils.hostread import landed
            cdev = landed(ch[0], ch[1]).copy()
            hmark("cols_synced")
        else:
            cdev = pre["cols_dev"].cpu().numpy()
        hmark("stack_checked")
        if cols is None or not np.array_equal(cdev, np.asarray(cols, dtype=np.int64)):
            if pre.get("speculative"):
                # the CV chose another alpha than the speculated one, with another selection: the
                # stack enqueued on the speculated columns is discarded and the fit redone
                LAST_PRELAUNCH["spec_miss"] = LAST_PRELAUNCH.get("spec_miss", 0) + 1
            else:
                import warnings
                warnings.warn("device column selection differs from the host's; relaunching the stacking fit")
            pre = None
    LAST_PRELAUNCH["used"] = pre is not None
    if pre is not None and pre.get("finished"):
        return clf          # (finish_prelaunched already completed it)
    if pre is not None:
        stc = pre["state"]
        stc["timer"] = timer or stc["timer"]
    else:
        stc = launch_stacking(clf, X, y, timer, group, svc_group, plan)
    return finish_stacking(stc)

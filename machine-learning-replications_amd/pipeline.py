"""End-to-end model development (reference ``train_ensemble_public.py:33-90``).

``develop(X_dev, y_dev, X_sel, y_sel, names)``:
KNN-impute (fit on dev, applied to both) → LassoCV/SelectFromModel top-17 →
stacking fit on dev → held-out ``predict_proba`` → report / AUROC / AP (+ plots).
Every step runs on the tensors' device; with ``group`` the dev rows are sharded
across ranks (see :mod:`hfens.parallel`).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from .config import EnsembleConfig, build_estimators, build_selector
from .models.imputer import KNNImputer
from .utils import metrics
from .utils.timing import StageTimer


# Multi-process policy for the stacking fit:
#   "dp"   — rows stay sharded; LassoCV moments, GBDT int64 histograms and LR Newton moments are
#            all-reduced every step, the SVC fits are spread over ranks.
#   "task" — after the (sharded) KNN imputation the imputed development rows are all-gathered
#            once; every rank then runs the cheap, latency-bound fits (LassoCV, GBDT, L1-LR, meta)
#            on the full rows itself and only the 36 SMO problems — the critical path — are
#            spread over the ranks (one SUM all-reduce of the solutions).  Identical results to a
#            single process, three collectives per fit instead of hundreds.
#   "auto" — task below HFENS_TASK_MAX_ROWS development rows (small data: the DP collectives'
#            latency exceeds the compute they split), dp above.
DP_POLICY = os.environ.get("HFENS_DP_POLICY", "auto")
TASK_MAX_ROWS = int(os.environ.get("HFENS_TASK_MAX_ROWS", str(1 << 18)))
AUX_STREAM = os.environ.get("HFENS_AUX_STREAM", "1") != "0"   # held-out imputation on a side stream
PLAN_AHEAD = os.environ.get("HFENS_PLAN_AHEAD", "1") != "0"   # stacking bookkeeping under the LassoCV path
# … computed on a host thread of its own: measured 32.3 vs 20.4 ms / fit (r5v) — the thread holds the
# GIL for up to the interpreter's switch interval each time the launching thread wakes from a device
# wait, so the launches behind it slip; off by default
PLAN_THREAD = os.environ.get("HFENS_PLAN_THREAD", "0") == "1"
# the GBC's bin map of every candidate column fitted on the host under the LassoCV path (the selected
# columns' bins are then a slice: binning.BinMapper.select), from one non-blocking copy of the imputed rows
# (default off: the GBC's host bin fit runs while the device solves the SVC, off the critical path)
BIN_AHEAD = os.environ.get("HFENS_BIN_AHEAD", "0") == "1"
INIT_STREAMS = os.environ.get("HFENS_INIT_STREAMS", "1") != "0"   # runtime.init_fit_streams
# the prelaunched stack's GBC / LR batches enqueued after the LassoCV's CV paths (1) or right behind
# the SVC batch, before the grid read (0, default).  Measured on one box (profiles/r6_runs/r6e): with
# the CV paths launched first, the paths, the SMO and the GBC stage loop ran side by side and the SMO
# took 15.5 instead of 11 ms (24.9 / 26.9 vs 19.0 / 18.6 ms / fit)
BASES_AFTER_CV = os.environ.get("HFENS_BASES_AFTER_CV", "0") == "1"
# the prelaunched stack finished (its host reads) before the LassoCV's own tail (its host reads of the
# CV paths' winner) instead of after it.  Measured slower (profiles/r6_runs/r6s: 18.9 / 18.7 vs
# 18.3 / 17.9 ms): the paths end ≈ 3 ms before the SMO, and their short tail then waited behind the
# stack's reads; off by default
FINISH_BEFORE_LASSO = os.environ.get("HFENS_FINISH_BEFORE_LASSO", "0") == "1"
# the native stacking plan (stack_trainer.plan_stacking_start, a helper thread with the GIL released)
# joined as the first job under the LassoCV's early speculation instead of right after the imputation
# is enqueued: the thread then has the LassoCV prelude's host time to finish in, and the join no
# longer waits for it on the host path to the SVC's cascade parts
PLAN_JOIN_LATE = os.environ.get("HFENS_PLAN_JOIN_LATE", "1") == "1"


def _bins_ahead(X_dev: torch.Tensor, clf):
    """Enqueue the float32 copy of the imputed development rows to pinned host memory on a side
    stream and return ``run()`` → the host bin fit of all columns (or None when the stack has no
    gradient-boosting member).  ``run`` waits only for that copy."""
    from .models.gbdt import GradientBoostingClassifier
    mb = [int(e.max_bins) for _, e in clf.estimators if isinstance(e, GradientBoostingClassifier)]
    if not mb or X_dev.shape[0] > (1 << 15):
        return None
    from . import runtime
    dev = X_dev.device
    # (the held-out imputation's side stream, ahead of that imputation: a stream of its own would
    # shift HIP's stream → hardware-queue round robin for every stream created after it — measured:
    # an extra stream here put the stacking trainer's streams on shared queues and cost the SMO 5 ms)
    side = runtime.stream(dev, "aux")
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        x32 = X_dev.to(torch.float32)
        xh = torch.empty(x32.shape, dtype=torch.float32, pin_memory=True)
        xh.copy_(x32, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(side)
    X_dev.record_stream(side)
    box = {}

    def run():
        if "bm" not in box:
            from .models.binning import fit_bins_host
            ev.synchronize()
            # (the bin tables' uploads are non-blocking copies on the side stream: on the current
            # stream they would queue behind the LassoCV path)
            with torch.cuda.stream(side):
                box["bm"] = fit_bins_host(xh.numpy(), mb[0], dev, non_blocking=True)
            box["ev"] = torch.cuda.Event()
            box["ev"].record(side)
        return box["bm"], box["ev"]
    return run


def choose_policy(n_total: int) -> str:
    if DP_POLICY in ("dp", "task"):
        return DP_POLICY
    return "task" if n_total <= TASK_MAX_ROWS else "dp"


@dataclass
class DevelopResult:
    model: object
    selected: np.ndarray
    selected_names: List[str]
    proba_sel: torch.Tensor
    report: str
    scores: Dict[str, float]
    timer: StageTimer
    n_train: int = 0


def develop(X_dev, y_dev, X_sel, y_sel, names, device="cpu", cfg: Optional[EnsembleConfig] = None,
            timer: Optional[StageTimer] = None, group=None, evaluate: bool = True) -> DevelopResult:
    cfg = cfg or EnsembleConfig()
    timer = timer or StageTimer(enabled=True, device=device if str(device).startswith("cuda") else None)
    dev = torch.device(device)
    X_dev = torch.as_tensor(np.asarray(X_dev) if not isinstance(X_dev, torch.Tensor) else X_dev,
                            dtype=torch.float64).to(dev)
    y_dev = torch.as_tensor(np.asarray(y_dev) if not isinstance(y_dev, torch.Tensor) else y_dev,
                            dtype=torch.float64).to(dev)
    X_sel = torch.as_tensor(np.asarray(X_sel) if not isinstance(X_sel, torch.Tensor) else X_sel,
                            dtype=torch.float64).to(dev)
    y_sel = torch.as_tensor(np.asarray(y_sel) if not isinstance(y_sel, torch.Tensor) else y_sel,
                            dtype=torch.float64).to(dev)
    if dev.type == "cuda" and INIT_STREAMS:
        from . import runtime
        runtime.init_fit_streams(dev)
    task = False
    if group is not None:
        from .parallel import dist as pdist
        task = choose_policy(pdist.all_reduce_int(X_dev.shape[0], group)) == "task"
    clf = build_estimators(cfg)
    # the stacking fit's label-only bookkeeping (folds, SVC problem expansions, Platt column maps)
    # is computed on the host while the LassoCV path runs on the device (stack_trainer.plan_stacking);
    # the labels come over in a non-blocking copy issued now, long finished by then
    plan_box = {}
    overlap = None

    def plan_ahead(y_full):
        # (task policy: called after the all-gather, so every rank plans from the same full labels)
        y_pin = torch.empty(y_full.shape[0], dtype=torch.float64, pin_memory=True)
        y_pin.copy_(y_full, non_blocking=True)
        y_ev = torch.cuda.Event()
        y_ev.record()

        box = {}
        native = None
        if not PLAN_THREAD:
            # the label work natively on a helper thread (GIL released) while this thread launches
            # the imputation and the LassoCV prelude; the labels' copy is done at once (idle device)
            from .models.stack_trainer import plan_stacking_start
            y_ev.synchronize()
            native = plan_stacking_start(clf, y_pin.numpy().copy())

        def work():
            try:
                from .models.stack_trainer import plan_stacking
                if native is not None:
                    box["plan"] = native()
                    return
                y_ev.synchronize()
                box["plan"] = plan_stacking(clf, y_pin.numpy().copy())
            except BaseException as e:   # re-raised by run() on the calling thread
                box["err"] = e

        if PLAN_THREAD:
            # on a host thread of its own: it runs while this thread waits on the device (the
            # imputation, LassoCV's prelude reads), not after
            import threading
            th = threading.Thread(target=work, name="hfens-plan", daemon=True)
            th.start()
        else:
            th = None

        def run():
            if th is not None:
                th.join()
            else:
                work()
            if "err" in box:
                raise box["err"]
            plan_box["plan"] = box["plan"]
        run.native = native is not None
        return run

    y_full = None
    if group is None and dev.type == "cuda" and PLAN_AHEAD:
        overlap = plan_ahead(y_dev)
    elif task:
        # the labels are gathered first (they do not wait for the imputation), so the plan below
        # is computed on the host while the device imputes, as in one process
        y_full = pdist.all_gather_rows(y_dev[:, None], group)[:, 0]
        if dev.type == "cuda" and PLAN_AHEAD:
            overlap = plan_ahead(y_full)
    from .utils.timing import hmark, dmark, dmarks_flush
    hmark("develop")
    dmark("develop")
    with timer.stage("impute"):
        if group is None:
            imputer = KNNImputer(n_neighbors=cfg.knn_neighbors).fit(X_dev)
        else:
            imputer = KNNImputer(n_neighbors=cfg.knn_neighbors).fit(pdist.all_gather_rows(X_dev, group))
        # this rank's rows (the O(n²) donor search is sharded) and the held-out rows, planned from
        # ONE host read; the held-out rows are only needed for the evaluation, so on the GPU
        # their donor search runs on a side stream, overlapped with LassoCV and the stacking fit
        # (joined before the evaluation below)
        aux = None
        if dev.type == "cuda" and AUX_STREAM:
            from . import runtime
            aux = runtime.stream(dev, "aux")
        hmark("imputer_fit")
        run_sel = None
        if aux is not None and (group is None or task):
            # the held-out rows' planning and launch (host numpy, ≈ 1 ms at 10k rows) are deferred
            # into the LassoCV path's device time below, off the host's critical path
            (X_dev, _), run_sel = imputer.transform_many([X_dev, X_sel], streams=[None, aux], defer=True)
        else:
            X_dev, X_sel = imputer.transform_many([X_dev, X_sel], streams=[None, aux])
        hmark("impute_enqueued")
        bins_job = _bins_ahead(X_dev, clf) if (BIN_AHEAD and dev.type == "cuda" and group is None) else None
        if task:
            X_dev = pdist.all_gather_rows(X_dev, group)
            y_dev = y_full
    fit_group = None if task else group
    sel = build_selector(cfg)
    planned = False
    # (task policy: every rank holds every row, so the single-process critical path applies — the
    # plan, the speculative LassoCV refit and the stacking prelaunch; only the SMO problems are
    # spread over the ranks, by the one all-reduce inside the prelaunched SVC batch)
    local = group is None or task
    if overlap is not None and local and not PLAN_THREAD and not (PLAN_JOIN_LATE and getattr(overlap, "native", False)):
        # the label-only stacking plan now, on the host, while the device imputes (LassoCV's
        # prelude reads wait for the imputation anyway): it is ready before the LassoCV path is
        # launched, so the stacking fit can be enqueued first thing under the path
        overlap()
        hmark("plan_ready")
        overlap, planned = None, True
    elif overlap is not None and local:
        # (PLAN_THREAD / a native plan with PLAN_JOIN_LATE: joined as the first job under the
        # LassoCV path)
        planned = True
    with timer.stage("select"):
        jobs, early_jobs = [], []
        held_out = None
        if run_sel is not None:
            def held_out():
                run_sel()
                hmark("heldout_impute_enqueued")
        if overlap is not None:
            early_jobs.append(overlap)
        if bins_job is not None:
            def bins():
                plan_box["bins_all"] = bins_job()
                hmark("bins_ahead")
            jobs.append(bins)
        if local and dev.type == "cuda" and (overlap is not None or planned):
            def stack_early():
                # the stacking fit (SVC batch, GBC / L1-LR batches, meta model) enqueued from the
                # selector's DEVICE column list — speculative (lasso.SPECULATE: the smallest-alpha
                # refit's selection, enqueued before the LassoCV's grid read, lasso.EARLY_SPEC) —
                # while the device still imputes / runs the LassoCV path (stack_trainer.prelaunch_stack)
                cols = getattr(sel, "cols_dev_", None)
                if cols is not None and plan_box.get("plan") is not None:
                    from .models.stack_trainer import prelaunch_stack
                    pre = prelaunch_stack(clf, X_dev, cols, y_dev, plan_box["plan"],
                                          svc_group=group if task else None)
                    if pre is not None:
                        pre["speculative"] = bool(getattr(sel, "cols_speculative_", False))
                        pre["cols_host"] = getattr(sel, "cols_host_", None)
                    plan_box["prelaunch"] = pre
            early_jobs.append(stack_early)
            def stack_bases():
                # the GBC / L1-LR batches and the meta model of the prelaunched stack, behind the
                # LassoCV's CV paths (which the speculation's check waits for)
                from .models.stack_trainer import prelaunch_bases
                prelaunch_bases(plan_box.get("prelaunch"))
                hmark("bases_prelaunched")
            if BASES_AFTER_CV:
                jobs.insert(0, stack_bases)
            else:
                early_jobs.append(stack_bases)
        if held_out is not None:
            jobs.append(held_out)     # (after the stacking fit: the held-out rows are needed last)

        def run_all(js):
            if not js:
                return None

            def f():
                for j in js:
                    j()
            return f
        tails = [] if (local and dev.type == "cuda" and planned and FINISH_BEFORE_LASSO) else None
        sfm = sel.fit(X_dev, y_dev, group=fit_group, overlap=run_all(jobs), early_overlap=run_all(early_jobs),
                      tail_out=tails)
        if tails:
            # the LassoCV fit returned with its CV paths still running: finish the stacking fit
            # enqueued on the speculative selection first (its host reads wait for the SMO), then
            # the LassoCV (its reads wait for the paths) — the host waits for both at once instead
            # of one after the other; fit_stacking checks the selection and redoes the stack on a miss
            pre = plan_box.get("prelaunch")
            if pre is not None:
                from .models.stack_trainer import finish_prelaunched
                finish_prelaunched(pre, timer)
                hmark("stack_spec_finished")
            for t in tails:
                t()
        if run_sel is not None:
            X_sel = run_sel()[1]      # (already run inside the LassoCV path; a no-op then)
        hmark("lasso_fit")
        dmark("lasso_fit")
        mask = sfm.get_support()
        mt = torch.as_tensor(mask, device=dev)
        X_dev_optm = X_dev[:, mt]
        fn_new = [n for n, m in zip(names, mask) if m]
        hmark("selected")
    plan = plan_box.get("plan")
    if plan_box.get("prelaunch") is not None:
        plan = dict(plan, prelaunch=plan_box["prelaunch"], cols=np.nonzero(mask)[0])
    if "bins_all" in plan_box:
        bm_all, bm_ev = plan_box["bins_all"]
        torch.cuda.current_stream(dev).wait_event(bm_ev)
        plan = dict(plan or {}, bins_all=bm_all, cols=np.nonzero(mask)[0])
    clf.fit(X_dev_optm, y_dev, timer=timer, group=fit_group, svc_group=group if task else None,
            plan=plan)
    dmark("stack_fit")
    hmark("stack_fit")
    if aux is not None:
        # join the side stream while the imputer and X_sel are alive (their blocks are not reused
        # by the main stream before this point)
        torch.cuda.current_stream(dev).wait_stream(aux)
    X_sel_optm = X_sel[:, mt]
    proba = None
    report = ""
    scores: Dict[str, float] = {}
    if evaluate:
        with timer.stage("predict_select"):
            proba = clf.predict_proba(X_sel_optm)[:, 1]
        yy = (proba > 0.5).to(torch.float64)
        if group is not None:
            from .parallel import dist as pdist
            proba_all = pdist.all_gather_rows(proba[:, None], group)[:, 0]
            ysel_all = pdist.all_gather_rows(y_sel[:, None], group)[:, 0]
            yy_all = (proba_all > 0.5).to(torch.float64)
        else:
            proba_all, ysel_all, yy_all = proba, y_sel, yy
        report = metrics.classification_report(ysel_all, yy_all)
        # (the held-out rows are already gathered for the report, so the AUROC comes from them;
        # metrics.roc_auc_sharded is the R8 path for callers that keep scores sharded)
        scores = metrics.evaluate(ysel_all, proba_all)
    hmark("develop_end")
    dmarks_flush()
    n_train = X_dev.shape[0]
    if fit_group is not None:
        from .parallel import dist as pdist
        n_train = pdist.all_reduce_int(n_train, group)
    return DevelopResult(clf, mask, fn_new, proba, report, scores, timer, n_train)

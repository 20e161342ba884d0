"""LassoCV + SelectFromModel feature selection (reference
``train_ensemble_public.py:51-55``: ``LassoCV(random_state=2020, cv=10)`` inside
``SelectFromModel(threshold=-inf, max_features=17)``).

Semantics (sklearn ``linear_model/_coordinate_descent.py``): a 100-alpha
geometric grid from ``max|Xcᵀyc|/n`` down to ``1e-3×`` that, 10 unshuffled KFold
folds, per fold a warm-started cyclic coordinate-descent path on the fold's
centred Gram matrix with the duality-gap stop (``tol·‖y‖²``), test MSE per alpha,
best alpha = argmin of the fold-mean MSE, refit on all rows at that alpha.
All 10 paths (+ the refit) run in the ``lasso_cd_path`` kernel, one wave per
fold; the Gram matrices come from one batched GEMM.  With a process group the
per-fold Gram / Xᵀy / yᵀy / row counts are all-reduced (rows sharded).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .base import Estimator, as_tensor
from .model_selection import kfold_test_folds


def _cd_path_host(G, q, yy, n, alphas, max_iter, tol):
    """numpy mirror of the lasso_cd_path kernel (one problem)."""
    F = G.shape[0]
    w = np.zeros(F)
    H = np.zeros(F)
    out = np.zeros((len(alphas), F))
    tol_s = tol * yy
    diag = np.diag(G)
    inv = np.where(diag != 0.0, 1.0 / np.where(diag != 0.0, diag, 1.0), 0.0)   # as the kernel: × 1/G_kk
    for a, alpha in enumerate(alphas):
        l1 = alpha * n
        for it in range(max_iter):
            w_max = d_w_max = 0.0
            for k in range(F):
                gkk = G[k, k]
                if gkk == 0.0:
                    continue
                tmp = q[k] - H[k] + gkk * w[k]
                nw = np.sign(tmp) * (abs(tmp) - l1) * inv[k] if abs(tmp) > l1 else 0.0
                dw = nw - w[k]
                if dw != 0.0:
                    H += G[:, k] * dw
                    w[k] = nw
                d_w_max = max(d_w_max, abs(dw))
                w_max = max(w_max, abs(nw))
            if w_max == 0.0 or d_w_max / w_max < tol or it == max_iter - 1:
                wq = w @ q
                dual = np.abs(q - H).max()
                R2 = yy - 2 * wq + w @ H
                const = 1.0
                gp = R2
                if dual > l1:
                    const = l1 / dual
                    gp = 0.5 * (R2 + R2 * const * const)
                gap = gp + l1 * np.abs(w).sum() - const * (yy - wq)
                if gap < tol_s:
                    break
        out[a] = w
    return out


SPECULATIVE_REFIT = os.environ.get("HFENS_LASSO_SPEC_REFIT", "1") != "0"
# Speculative selection (device path): the CV paths run on a stream of their own, and beside them one
# cold-start solve on all rows at the grid's SMALLEST alpha — the refit the CV choice makes whenever
# the least-regularised model wins (on the Table S1-shaped cohorts it does: best = last of 100 alphas
# on three draws).  Its coefficients (``coef_spec_dev_``, event ``spec_ev_``) are ready long before the
# CV paths end, so a caller's overlap can start work on the selection they imply (the stacking
# trainer's SVC batch) while the paths still run; the caller checks the speculation against the real
# selection afterwards and redoes the work on a miss.  The CV-side results are computed after the
# overlap, so nothing the overlap enqueues waits behind the paths.
SPECULATE = os.environ.get("HFENS_LASSO_SPECULATE", "1") != "0"
SPEC_ALPHA_INDEX = -1     # the grid point speculated on (tests move it to force a miss)
EARLY_SPEC = os.environ.get("HFENS_LASSO_EARLY_SPEC", "1") != "0"
# with the early speculation, the every-alpha refit beside the CV paths is not solved (the hit's refit
# is the speculative one; a miss solves its one refit after the paths): its 100 one-wave solves ran
# beside the prelaunched stack and held CUs the GBDT stage kernel and the SMO needed
# (profiles/r6_runs/r6d: 25.2 vs 19.2 ms / fit with the bases behind the paths)
EARLY_REFIT_ALL = os.environ.get("HFENS_LASSO_EARLY_REFIT_ALL", "0") == "1"


class LassoCV(Estimator):
    _param_names = ("eps", "n_alphas", "alphas", "fit_intercept", "max_iter", "tol", "cv", "random_state",
                    "selection")

    def __init__(self, eps=1e-3, n_alphas=100, alphas=None, fit_intercept=True, max_iter=1000, tol=1e-4,
                 cv=None, random_state=None, selection="cyclic"):
        self.eps = eps
        self.n_alphas = n_alphas
        self.alphas = alphas
        self.fit_intercept = fit_intercept
        self.max_iter = max_iter
        self.tol = tol
        self.cv = cv
        self.random_state = random_state
        self.selection = selection

    def _solve(self, Gs, qs, yys, ns, alpha_grid):
        """Run P coordinate-descent paths; Gs [P,F,F], qs [P,F], alpha_grid [P,A]."""
        P, F = qs.shape
        A = alpha_grid.shape[1]
        if Gs.is_cuda and F <= 64:
            from .. import ops
            E = ops.ext()
            coefs = torch.empty(P, A, F, dtype=torch.float64, device=Gs.device)
            gaps = torch.empty(P, A, dtype=torch.float64, device=Gs.device)
            iters = torch.empty(P, A, dtype=torch.int32, device=Gs.device)
            E.lasso_cd_path(P, F, A, Gs.contiguous().data_ptr(), qs.contiguous().data_ptr(),
                            yys.contiguous().data_ptr(), ns.contiguous().data_ptr(),
                            alpha_grid.contiguous().data_ptr(), int(self.max_iter), float(self.tol),
                            coefs.data_ptr(), gaps.data_ptr(), iters.data_ptr(), ops.stream_ptr(Gs.device))
            return coefs
        out = [torch.as_tensor(_cd_path_host(Gs[p].cpu().numpy(), qs[p].cpu().numpy(), float(yys[p]),
                                             float(ns[p]), alpha_grid[p].cpu().numpy(), int(self.max_iter),
                                             float(self.tol))) for p in range(P)]
        return torch.stack(out).to(Gs.device)

    def fit(self, X, y, group=None, overlap=None, early_overlap=None, tail_out=None):
        """``overlap``: optional host callable run while the device solves the CV path (between its
        launch and the first read of its result) — host work hidden under the path's GPU time.
        ``early_overlap``: run right after the speculative refit is enqueued, before the alpha grid's
        host read (only when the speculation runs early, :data:`EARLY_SPEC`).  ``tail_out`` (a list,
        early speculation only): the fit returns once the CV paths are enqueued and appends the
        closure that completes it (waits for the paths, picks α, refits) — the caller runs it later."""
        from ..utils.guards import check_finite, finite_flag, raise_flags
        X = as_tensor(X)
        y = as_tensor(y, device=X.device)
        dev = X.device
        one_read = dev.type == "cuda" and group is None and self.alphas is None
        if one_read:
            # the input guards ride on the alpha grid's read below (ONE host read in the prelude)
            flags = [finite_flag(X), finite_flag(y)]
        else:
            check_finite(X, "LassoCV.fit X")
            check_finite(y, "LassoCV.fit y")
        n, F = X.shape
        k = 5 if self.cv is None else int(self.cv)
        if group is None:
            tfh = torch.from_numpy(kfold_test_folds(n, k))
            # (pinned, non-blocking: a pageable upload waits for the stream's queued work)
            tf = tfh.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else tfh.to(dev)
        else:
            from ..parallel import dist as pdist
            tf = pdist.sharded_kfold_test_folds(n, k, group, dev)
        # per-fold training moments (rows in fold f are excluded from problem f) + full data
        masks = torch.stack([tf != f for f in range(k)] + [torch.ones(n, dtype=torch.bool, device=dev)])
        mk = masks.to(torch.float64)                         # [P, n]
        cnt = mk.sum(1)
        sy = mk @ y
        Syy = mk @ (y * y)
        from .. import ops
        Sxx, sx, Sxy = ops.weighted_moments(X, mk, mk * y[None])   # one reduction kernel
        if group is not None:
            from ..parallel import dist as pdist
            cnt, sx, sy, Sxx, Sxy, Syy = pdist.all_reduce_sum_f64([cnt, sx, sy, Sxx, Sxy, Syy], group)
        mx = sx / cnt[:, None]
        my = sy / cnt
        G = Sxx - cnt[:, None, None] * mx[:, :, None] * mx[:, None, :]
        q = Sxy - cnt[:, None] * mx * my[:, None]
        yy = Syy - cnt * my * my
        from ..utils.timing import dmark, hmark
        main = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
        self.coef_spec_dev_ = self.spec_ev_ = None
        # (only a caller with an overlap can use the speculation: SelectFromModel's)
        spec = (dev.type == "cuda" and F <= 64 and SPECULATIVE_REFIT and SPECULATE and group is None
                and overlap is not None)
        # EARLY_SPEC: the speculative refit goes in BEFORE the alpha grid's host read (which waits for
        # the imputation): np.geomspace's end points are exactly amax and amax·eps (numpy assigns them),
        # and amax = max|q| / n is one IEEE division, so the device computes the speculated grid
        # point bit for bit.  The caller's early overlap (the stacking fit enqueued on the speculative
        # selection) then runs while the device still imputes, instead of after the read.
        early = (spec and EARLY_SPEC and self.alphas is None and one_read
                 and SPEC_ALPHA_INDEX % self.n_alphas in (0, self.n_alphas - 1))
        if early:
            res = float(np.finfo(np.float64).resolution)
            amax_d = q[k].abs().max() / cnt[k]
            a_d = amax_d if SPEC_ALPHA_INDEX % self.n_alphas == 0 else amax_d * self.eps
            a_d = torch.where(amax_d <= res, torch.full_like(a_d, res), a_d)
            # (on the caller's stream: its consumers — the speculative selection and the stacking
            # batches enqueued on it — wait for it anyway; the CV paths below start behind it)
            self.coef_spec_dev_ = self._solve(G[k:], q[k:], yy[k:], cnt[k:], a_d.reshape(1, 1))[0, 0]
            dmark("lasso_spec")
            self.spec_ev_ = torch.cuda.Event()
            self.spec_ev_.record(main)
            self.spec_alpha_dev_ = a_d
            if early_overlap is not None:
                hmark("lasso_spec_launched")
                early_overlap()
        # alpha grid on all rows (problem k = full data)
        if self.alphas is None:
            if one_read:
                hv = torch.stack([q[k].abs().max(), cnt[k], flags[0].to(torch.float64),
                                  flags[1].to(torch.float64)]).cpu().tolist()
                raise_flags([hv[2] != 0.0, hv[3] != 0.0], [("finite", "LassoCV.fit X"), ("finite", "LassoCV.fit y")])
                amax = hv[0] / hv[1]
            else:
                amax = float(q[k].abs().max()) / float(cnt[k])
            if amax <= np.finfo(np.float64).resolution:
                grid = torch.full((self.n_alphas,), np.finfo(np.float64).resolution, dtype=torch.float64)
            else:
                grid = torch.as_tensor(np.geomspace(amax, amax * self.eps, num=self.n_alphas))
        else:
            grid = torch.as_tensor(np.sort(np.asarray(self.alphas, dtype=np.float64))[::-1].copy())
        grid = grid.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else grid.to(dev)
        A = int(grid.numel())
        refit_all = None
        if spec and not early:
            from .. import runtime
            sst = runtime.stream(dev, "lasso_spec", priority=-1)
            sst.wait_stream(main)
            with torch.cuda.stream(sst):
                # (the same kernel on the same inputs as refit_all's last problem: bit-identical)
                a = SPEC_ALPHA_INDEX % A
                self.coef_spec_dev_ = self._solve(G[k:], q[k:], yy[k:], cnt[k:], grid[a:a + 1][None])[0, 0]
                dmark("lasso_spec")
                self.spec_ev_ = torch.cuda.Event()
                self.spec_ev_.record(sst)
            for t in (G, q, yy, cnt, grid):
                t.record_stream(sst)     # (the solve may still read them after fit returns)
        if early:
            # the CV paths, then every alpha's cold-start refit (below), on ONE side stream: neither
            # is on the critical path any more (the stacking fit already runs on the speculative
            # selection), and no further stream changes the measured stream → hardware-queue layout
            from .. import runtime
            pst = runtime.stream(dev, "lasso_refit")
            pst.wait_stream(main)
            with torch.cuda.stream(pst):
                coefs = self._solve(G[:k], q[:k], yy[:k], cnt[:k], grid[None].expand(k, -1))   # [k, A, F]
                dmark("lasso_cv_path")
                path_ev = torch.cuda.Event()
                path_ev.record(pst)
            coefs.record_stream(main)
        if dev.type == "cuda" and F <= 64 and SPECULATIVE_REFIT and not (early and not EARLY_REFIT_ALL):
            # the refit at the CV-chosen alpha is a cold-start solve on all rows (sklearn's
            # Lasso(alpha=best).fit); which alpha wins is known only after the CV paths, so solve the
            # cold start for EVERY alpha on a side stream while the CV paths run (one wave each, the
            # device is otherwise idle) and pick the winner afterwards: the same kernel on the same
            # inputs as the one-problem refit, bit-identical, and no second dependent launch on the
            # critical path
            from .. import runtime
            side = runtime.stream(dev, "lasso_refit")
            side.wait_stream(main)
            with torch.cuda.stream(side):
                refit_all = self._solve(G[k:].expand(A, F, F), q[k:].expand(A, F), yy[k:].expand(A),
                                        cnt[k:].expand(A), grid[:, None])          # [A, 1, F]
                ev = torch.cuda.Event()
                ev.record(side)
        dmark("lasso_cv_in")
        join_ev = None
        if early:
            for t in (G, q, yy, cnt, grid):
                t.record_stream(pst)
            if overlap is not None:
                hmark("lasso_launched")
                overlap()
                overlap = None
            join_ev = path_ev      # (joined in tail(): the MSE below waits for the paths)
        elif spec:
            # the CV paths on a stream of their own: work the overlap enqueues on the caller's stream
            # does not queue behind them (joined before the MSE below, after the overlap)
            pst = runtime.stream(dev, "lasso_path")
            pst.wait_stream(main)
            with torch.cuda.stream(pst):
                coefs = self._solve(G[:k], q[:k], yy[:k], cnt[:k], grid[None].expand(k, -1))   # [k, A, F]
                dmark("lasso_cv_path")
                path_ev = torch.cuda.Event()
                path_ev.record(pst)
            for t in (G, q, yy, cnt, grid):
                t.record_stream(pst)
            coefs.record_stream(main)
            if overlap is not None:
                hmark("lasso_launched")
                overlap()
                overlap = None
            main.wait_event(path_ev)
        else:
            coefs = self._solve(G[:k], q[:k], yy[:k], cnt[:k], grid[None].expand(k, -1))   # [k, A, F]
            dmark("lasso_cv_path")
        def tail():
            """The CV paths' winner, its refit and the fitted attributes (the host reads)."""
            nonlocal overlap
            if join_ev is not None:
                main.wait_event(join_ev)
            hmark("lasso_tail")
            # test MSE per fold and alpha: residual = X_test·w + (ȳ_tr − x̄_tr·w) − y_test
            inter = my[:k, None] - torch.einsum("pf,paf->pa", mx[:k], coefs)               # [k, A]
            # Σ_test (x·w + c − y)² from the test-fold moments (all rows minus fold-train rows);
            # already globally reduced, so no per-row pass and no [k, A, n] intermediate.
            Txx, Tx, Txy = Sxx[k] - Sxx[:k], sx[k] - sx[:k], Sxy[k] - Sxy[:k]
            Ty, Tyy, nt = sy[k] - sy[:k], Syy[k] - Syy[:k], cnt[k] - cnt[:k]
            c = inter
            se = (torch.einsum("paf,pfg,pag->pa", coefs, Txx, coefs)
                  + 2 * c * torch.einsum("pf,paf->pa", Tx, coefs) - 2 * torch.einsum("pf,paf->pa", Txy, coefs)
                  + nt[:, None] * c * c - 2 * c * Ty[:, None] + Tyy[:, None])
            mse = se / nt[:, None]                                                          # [k, A]
            mean_mse = mse.mean(0)
            best_dev = torch.argmin(mean_mse)
            self.coef_dev_ = None
            if refit_all is not None:
                # the winner's coefficients stay on the device (no host read): a caller's overlap can
                # queue work that depends on them (SelectFromModel's device column list → the stacking
                # trainer's SVC batch) before this fit reads anything back
                torch.cuda.current_stream(dev).wait_event(ev)
                self.coef_dev_ = refit_all.index_select(0, best_dev.reshape(1))[0, 0]
            if overlap is not None:
                overlap()
            best = int(best_dev)
            hmark("lasso_best_read")
            self.alpha_ = float(grid[best])
            self.alphas_ = grid
            self.mse_path_ = mse.t()
            if refit_all is not None:
                w = refit_all[best, 0]
            elif (early and best == SPEC_ALPHA_INDEX % A
                  and float(self.spec_alpha_dev_) == float(grid[best])):
                # the speculation hit: its refit IS the refit at the chosen alpha (same kernel, same
                # inputs, the same alpha bits)
                w = self.coef_spec_dev_
            else:
                final = self._solve(G[k:], q[k:], yy[k:], cnt[k:], grid[best:best + 1][None])
                w = final[0, 0]
            self.coef_ = w
            self.intercept_ = my[k] - mx[k] @ w
            self.n_features_in_ = F
            return self

        if tail_out is not None and early:
            # the caller completes the fit later (pipeline.develop: after finishing the stacking fit
            # enqueued on the speculative selection, so the host waits for both at once)
            tail_out.append(tail)
            return self
        return tail()


class SelectFromModel(Estimator):
    """``SelectFromModel(estimator, threshold=-inf, max_features=k)``: keep the k
    largest |coef| (stable order), in original column order."""
    _param_names = ("estimator", "threshold", "max_features")

    def __init__(self, estimator, threshold=None, max_features=None):
        self.estimator = estimator
        self.threshold = threshold
        self.max_features = max_features

    def _device_columns(self, coef_dev: torch.Tensor, F: int):
        """The selected columns (ascending) from device coefficients, on the device: feature f is
        kept iff its rank in ``argsort(−|coef|, kind='mergesort')`` (ties: lower index first) is
        below max_features — the host rule of :meth:`fit` for threshold=-inf."""
        k = min(int(self.max_features), F)
        s = coef_dev.abs()
        idx = torch.arange(F, device=s.device)
        rank = ((s[None, :] > s[:, None]) | ((s[None, :] == s[:, None]) & (idx[None, :] < idx[:, None]))).sum(1)
        key = torch.where(rank < k, idx, idx + F)
        return torch.sort(key, stable=True).values[:k]

    def fit(self, X, y, group=None, overlap=None, early_overlap=None, tail_out=None):
        """``overlap`` / ``early_overlap``: host callables run under the LassoCV path (see
        :meth:`LassoCV.fit`).  With threshold=-inf and max_features, ``cols_dev_`` (the selected
        columns on the device, from the speculative refit when there is one) is set before either
        runs; ``early_overlap`` runs as soon as the speculative selection is enqueued (before the
        LassoCV's host read) or, without an early speculation, right before ``overlap``.
        ``tail_out``: see :meth:`LassoCV.fit` — the selection is then completed by the appended
        closure."""
        self.cols_dev_ = None
        self.cols_host_ = None
        if (overlap is not None or early_overlap is not None) and isinstance(self.estimator, LassoCV):
            user_late, user_early = overlap, early_overlap
            done = [False]
            dev_rule = (self.max_features is not None and isinstance(self.threshold, float)
                        and np.isneginf(self.threshold))

            def early():
                if done[0]:
                    return
                done[0] = True
                if dev_rule:
                    est = self.estimator
                    cd = getattr(est, "coef_spec_dev_", None)
                    self.cols_speculative_ = cd is not None
                    if cd is not None:
                        # speculative: the selection of the smallest-alpha refit (LassoCV.SPECULATE),
                        # checked against the real selection by whoever uses it
                        torch.cuda.current_stream(cd.device).wait_event(est.spec_ev_)
                    else:
                        cd = getattr(est, "coef_dev_", None)
                    if cd is not None:
                        self.cols_dev_ = self._device_columns(cd, int(cd.shape[0]))
                        # the host copy for the caller's check, read right behind the columns
                        # (pinned + event), on a pool stream
                        from .. import runtime
                        main = torch.cuda.current_stream(cd.device)
                        cs = runtime.stream(cd.device, "lasso_refit")
                        cs.wait_stream(main)
                        from ..utils.hostread import stage
                        with torch.cuda.stream(cs):
                            self.cols_host_ = stage(self.cols_dev_, cs)   # (polled: utils.hostread)
                        self.cols_dev_.record_stream(cs)
                    from ..utils.timing import hmark
                    hmark("cols_dev")
                if user_early is not None:
                    user_early()

            def late():
                early()
                if user_late is not None:
                    user_late()
            inner = [] if tail_out is not None else None
            self.estimator_ = self.estimator.fit(X, y, group=group, overlap=late, early_overlap=early,
                                                 tail_out=inner)
            if inner:
                def tail():
                    inner[0]()
                    self._select()
                tail_out.append(tail)
                return self
        else:
            self.estimator_ = self.estimator.fit(X, y, group=group)
            for f in (early_overlap, overlap):
                if f is not None:
                    f()
        return self._select()

    def _select(self):
        scores = self.estimator_.coef_.abs().cpu().numpy()
        F = scores.size
        mask = np.ones(F, dtype=bool)
        if self.threshold is not None and not (isinstance(self.threshold, float) and np.isneginf(self.threshold)):
            thr = float(np.mean(scores)) if self.threshold == "mean" else float(self.threshold)
            mask &= scores >= thr
        if self.max_features is not None:
            keep = np.zeros(F, dtype=bool)
            keep[np.argsort(-scores, kind="mergesort")[: int(self.max_features)]] = True
            mask &= keep
        self.support_ = mask
        return self

    def get_support(self) -> np.ndarray:
        return self.support_

    def transform(self, X):
        return X[:, torch.as_tensor(self.support_, device=X.device)]

"""KNN imputation (reference ``train_ensemble_public.py:37-40``:
``KNNImputer(missing_values=nan, n_neighbors=1)`` fit on the development set and
applied to both sets; semantics sklearn ``impute/_knn.py`` + ``nan_euclidean``).

For every missing cell (r, c) the donor is the fit row with column c present that
minimises the nan-euclidean distance ``F/|common|·Σ_common (x−y)²``; with no
defined distance the column mean of the fit rows is used.  Donor search runs in
the ``knn_donors`` HIP kernel (tie-break: lowest donor index; sklearn's
``argpartition`` tie order is unspecified).  ``n_neighbors > 1`` (uniform mean
over the k nearest) runs on the host path.
"""
from __future__ import annotations

import numpy as np
import torch

from .base import Estimator, as_tensor

SLOTS = 8


def _masks_u64(miss: torch.Tensor) -> torch.Tensor:
    F = miss.shape[1]
    w = (2 ** torch.arange(F, dtype=torch.int64, device=miss.device))
    bits = (miss.to(torch.int64) * w).sum(1)
    return bits


class KNNImputer(Estimator):
    _param_names = ("missing_values", "n_neighbors", "weights", "metric", "copy")

    def __init__(self, missing_values=np.nan, n_neighbors=5, weights="uniform", metric="nan_euclidean",
                 copy=True):
        self.missing_values = missing_values
        self.n_neighbors = n_neighbors
        self.weights = weights
        self.metric = metric
        self.copy = copy

    def fit(self, X):
        X = as_tensor(X)
        self._fit_X = X
        self._mask_fit = torch.isnan(X)
        self._valid = ~self._mask_fit.all(0)
        fx = torch.where(self._mask_fit, torch.zeros_like(X), X)
        cnt = (~self._mask_fit).sum(0).clamp(min=1)
        self._col_mean = fx.sum(0) / cnt
        return self

    def fit_transform(self, X):
        return self.fit(X).transform(X)

    def transform(self, X):
        X = as_tensor(X, device=self._fit_X.device).clone()
        miss = torch.isnan(X)
        rows = torch.nonzero(miss.any(1)).squeeze(1)
        if rows.numel() > 0:
            if X.is_cuda and self.n_neighbors == 1:
                self._impute_device(X, miss, rows)
            else:
                self._impute_host(X, miss, rows)
        return X[:, self._valid]

    # ------------------------------------------------------------------ device
    def _impute_device(self, X, miss, rows):
        from .. import ops
        E = ops.ext()
        F = X.shape[1]
        if F > 64:
            raise ValueError("KNNImputer device path supports at most 64 features")
        D = torch.where(self._mask_fit, torch.zeros_like(self._fit_X), self._fit_X)
        center = self._col_mean  # centring improves f32 accuracy; distances are shift-invariant
        D32 = (D - center).where(~self._mask_fit, torch.zeros_like(D)).to(torch.float32).contiguous()
        dm = _masks_u64(self._mask_fit).contiguous()
        Rm = miss[rows]
        R = torch.where(Rm, torch.zeros_like(X[rows]), X[rows] - center)
        R32 = R.to(torch.float32).contiguous()
        rm = _masks_u64(Rm).contiguous()
        nmiss = Rm.sum(1)
        order = torch.argsort((~Rm).to(torch.int8), dim=1, stable=True)   # missing columns first
        max_m = int(nmiss.max())
        for s0 in range(0, max_m, SLOTS):
            cols = order[:, s0:s0 + SLOTS]
            if cols.shape[1] < SLOTS:
                cols = torch.cat([cols, torch.zeros(cols.shape[0], SLOTS - cols.shape[1], dtype=cols.dtype,
                                                    device=cols.device)], 1)
            k = torch.arange(s0, s0 + SLOTS, device=X.device)
            valid = k[None, :] < nmiss[:, None]
            slot = torch.where(valid, cols, torch.full_like(cols, -1)).to(torch.int32).contiguous()
            best = torch.empty(slot.shape, dtype=torch.int64, device=X.device)
            E.knn_donors(R32.data_ptr(), rm.data_ptr(), rows.numel(), D32.data_ptr(), dm.data_ptr(),
                         D32.shape[0], F, slot.data_ptr(), best.data_ptr(), ops.stream_ptr(X.device))
            # packed (d² float bits << 32 | donor); all-ones = no donor with a defined distance
            donor = torch.where(best == -1, torch.full_like(best, -1), best & 0xFFFFFFFF)
            r_idx = rows[:, None].expand_as(slot)[valid]
            c_idx = slot[valid].long()
            donor = donor[valid]
            vals = torch.where(donor >= 0, self._fit_X[donor.clamp(min=0), c_idx], self._col_mean[c_idx])
            X[r_idx, c_idx] = vals

    # ------------------------------------------------------------------ host
    def _impute_host(self, X, miss, rows):
        fit = self._fit_X
        mf = self._mask_fit
        F = X.shape[1]
        D = torch.where(mf, torch.zeros_like(fit), fit)
        pres_f = (~mf).to(torch.float64)
        step = max(1, (1 << 24) // max(1, fit.shape[0] * F))
        for s in range(0, rows.numel(), step):
            rr = rows[s:s + step]
            R = X[rr]
            mr = torch.isnan(R)
            Rz = torch.where(mr, torch.zeros_like(R), R)
            pres_r = (~mr).to(torch.float64)
            # Σ_common (x−y)², direct differences in f64 (exact ties stay ties)
            both = pres_r[:, None, :] * pres_f[None, :, :]
            d2 = (both * (Rz[:, None, :] - D[None, :, :]) ** 2).sum(-1)
            common = both.sum(-1)
            dist = torch.where(common > 0, d2 * F / common.clamp(min=1),
                               torch.full_like(d2, float("inf")))
            for j, r in enumerate(rr.tolist()):
                for c in torch.nonzero(mr[j]).squeeze(1).tolist():
                    cand = ~mf[:, c]
                    dd = torch.where(cand, dist[j], torch.full_like(dist[j], float("inf")))
                    k = min(self.n_neighbors, int(cand.sum()))
                    if k == 0 or not torch.isfinite(dd).any():
                        X[r, c] = self._col_mean[c]
                        continue
                    if k == 1:
                        X[r, c] = fit[int(torch.argmin(dd)), c]   # first minimum = lowest index
                        continue
                    vals, idx = torch.topk(-dd, k)
                    ok = torch.isfinite(vals)
                    X[r, c] = fit[idx[ok], c].mean()

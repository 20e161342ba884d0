"""StandardScaler (reference ``train_ensemble_public.py:44``; semantics sklearn
``preprocessing/_data.py``: population variance, ``scale_ = sqrt(var_)`` with
zero variance mapped to 1)."""
from __future__ import annotations

import torch

from .base import Estimator, as_tensor


class StandardScaler(Estimator):
    _param_names = ("with_mean", "with_std", "copy")

    def __init__(self, with_mean=True, with_std=True, copy=True):
        self.with_mean = with_mean
        self.with_std = with_std
        self.copy = copy

    def fit(self, X, sample_mask=None):
        """Column moments in fp64 (K2 ``col_moments``); ``sample_mask`` selects rows."""
        X = as_tensor(X)
        if sample_mask is not None:
            X = X[sample_mask]
        n = X.shape[0]
        # Σx / n and Σ(x − mean)² / n with a TRUE division, as sklearn's _incremental_mean_and_var
        # (nansum / n, nanvar).  On the GPU, torch divides a tensor by a Python scalar as a multiply
        # by its reciprocal (measured: 14396.0 / 7198 → 1.9999999999999998), which turns a constant
        # column's variance into 5e-32 and its scale into 2e-16 instead of the exact 0 → 1 of the
        # 0.23.2 rule; dividing by a tensor of n is an IEEE division
        nt = torch.full((X.shape[1],), float(n), dtype=X.dtype, device=X.device)
        mean = X.sum(0) / nt
        var = ((X - mean) ** 2).sum(0) / nt
        self._set(mean, var, n)
        return self

    def _set(self, mean, var, n):
        self.n_features_in_ = int(mean.numel())
        self.n_samples_seen_ = int(n)
        self.mean_ = mean.to(torch.float64)
        self.var_ = var.to(torch.float64)
        scale = torch.sqrt(self.var_)
        # sklearn 0.23.2 (the checkpoint's version) ``_handle_zeros_in_scale`` maps only an exact
        # zero to 1; the ``< 10·eps`` rule is sklearn ≥ 1.0 and would rescale near-constant
        # columns (e.g. a binary flag nearly constant inside one CV fold) differently
        self.scale_ = torch.where(scale == 0.0, torch.ones_like(scale), scale)
        return self

    def _set_parts(self, mean, var, scale, n):
        """:meth:`_set` with the scale already formed (the stacking trainer forms every fold's scale
        in one batched sqrt / where — the same elementwise expressions)."""
        self.n_features_in_ = int(mean.numel())
        self.n_samples_seen_ = int(n)
        self.mean_, self.var_, self.scale_ = mean, var, scale
        return self

    def transform(self, X):
        X = as_tensor(X, device=self.mean_.device)
        if self.with_mean:
            X = X - self.mean_
        if self.with_std:
            X = X / self.scale_
        return X

    def fit_transform(self, X):
        return self.fit(X).transform(X)

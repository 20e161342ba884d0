"""Logistic regression: the L1/liblinear base model 'lg' and the L2/lbfgs meta
learner (reference ``train_ensemble_public.py:46,48``).

Solvers (device-resident, batched over many independent fits):

* ``penalty='l1'`` — liblinear's objective ``‖w‖₁ + C·Σ sw_i·log(1+e^{-y_i w·x̃_i})`` with
  the intercept folded in as an augmented feature (``intercept_scaling=1``), so the
  intercept is L1-penalised exactly as in liblinear.  Solved by a
  proximal-Newton / coordinate-descent method (newGLMNET-equivalent optimum).
* ``penalty='l2'`` — ``½‖w‖² + C·Σ sw_i·logloss_i`` with an unpenalised intercept,
  minimised by batched Newton (the lbfgs optimum).
"""
from __future__ import annotations

import torch

from .base import Estimator, as_tensor, balanced_class_weight


class LogisticRegression(Estimator):
    _param_names = ("penalty", "dual", "tol", "C", "fit_intercept", "intercept_scaling", "class_weight",
                    "random_state", "solver", "max_iter", "multi_class", "verbose", "warm_start",
                    "n_jobs", "l1_ratio")

    def __init__(self, penalty="l2", dual=False, tol=1e-4, C=1.0, fit_intercept=True,
                 intercept_scaling=1, class_weight=None, random_state=None, solver="lbfgs",
                 max_iter=100, multi_class="auto", verbose=0, warm_start=False, n_jobs=None,
                 l1_ratio=None):
        self.penalty = penalty
        self.dual = dual
        self.tol = tol
        self.C = C
        self.fit_intercept = fit_intercept
        self.intercept_scaling = intercept_scaling
        self.class_weight = class_weight
        self.random_state = random_state
        self.solver = solver
        self.max_iter = max_iter
        self.multi_class = multi_class
        self.verbose = verbose
        self.warm_start = warm_start
        self.n_jobs = n_jobs
        self.l1_ratio = l1_ratio
        # (framework option, not a scikit-learn parameter: never pickled) penalty='l1' +
        # solver='liblinear': reproduce liblinear's default-tolerance iterate and its seed draw
        # (logreg_solver._fit_liblinear_exact) instead of solving to the optimum on the device
        self.emulate_liblinear = False

    def clone(self):
        c = super().clone()
        c.emulate_liblinear = self.emulate_liblinear
        return c

    def sample_weights(self, y: torch.Tensor) -> torch.Tensor:
        if self.class_weight == "balanced":
            cw = balanced_class_weight(y)
            return cw[y.long()]
        return torch.ones_like(y, dtype=torch.float64)

    def fit(self, X, y, sample_mask=None):
        from .logreg_solver import fit_logreg_batch
        X = as_tensor(X)
        y = as_tensor(y, device=X.device)
        mask = None if sample_mask is None else sample_mask[None]
        fit_logreg_batch([self], X, y, mask)
        return self

    def decision_function(self, X) -> torch.Tensor:
        X = as_tensor(X, device=self.coef_.device)
        return X @ self.coef_[0] + self.intercept_[0]

    def predict_proba(self, X) -> torch.Tensor:
        p1 = torch.sigmoid(self.decision_function(X))
        return torch.stack([1 - p1, p1], dim=1)

    def predict(self, X) -> torch.Tensor:
        return (self.decision_function(X) > 0).to(torch.float64)

    def set_fitted(self, coef, intercept, n_iter, n_features, device=None):
        self.n_features_in_ = int(n_features)
        # (arange: a device fill, not a blocking host→device copy behind the stream's queued work)
        self.classes_ = torch.arange(2, dtype=torch.int64, device=device)
        self.coef_ = as_tensor(coef, device).reshape(1, -1)
        self.intercept_ = as_tensor(intercept, device).reshape(1)
        self.n_iter_ = as_tensor(n_iter, device, torch.int32).reshape(1)
        return self

"""Pipeline + StackingClassifier (reference ``train_ensemble_public.py:43-48,61-62``;
semantics sklearn ``ensemble/_stacking.py``: base models refit on all rows,
meta-features = out-of-fold ``predict_proba[:, 1]`` from StratifiedKFold(5),
meta learner fit on those).

Training is orchestrated as *batched* fits: the 5 OOF folds + the full refit of
each base model (6 fits) are solved together on the device — one histogram
launch sequence for the 6 GBDTs, one coordinate-descent launch for the 6 L1
logistic models, one SMO launch for the 36 SVM problems (6 SVC fits × (5 Platt
folds + 1)).  With a process group the fits are spread over ranks
(:mod:`hfens.parallel`).
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from .. import ops
from .base import Estimator, as_tensor


class Pipeline(Estimator):
    _param_names = ("steps", "memory", "verbose")

    def __init__(self, steps, memory=None, verbose=False):
        self.steps = list(steps)
        self.memory = memory
        self.verbose = verbose

    @property
    def named_steps(self):
        return dict(self.steps)

    def clone(self):
        return Pipeline([(n, s.clone()) for n, s in self.steps], self.memory, self.verbose)

    def _transform(self, X):
        for _, s in self.steps[:-1]:
            X = s.transform(X)
        return X

    def fit(self, X, y):
        for _, s in self.steps[:-1]:
            X = s.fit(X).transform(X)
        self.steps[-1][1].fit(X, y)
        return self

    def predict_proba(self, X):
        return self.steps[-1][1].predict_proba(self._transform(X))

    def decision_function(self, X):
        return self.steps[-1][1].decision_function(self._transform(X))

    def to(self, device):
        for _, s in self.steps:
            s.to(device)
        return self


def make_pipeline(*steps) -> Pipeline:
    return Pipeline([(type(s).__name__.lower(), s) for s in steps])


class StackingClassifier(Estimator):
    _param_names = ("estimators", "final_estimator", "cv", "stack_method", "n_jobs", "passthrough",
                    "verbose")

    def __init__(self, estimators, final_estimator=None, cv=None, stack_method="auto", n_jobs=None,
                 passthrough=False, verbose=0):
        self.estimators = list(estimators)
        self.final_estimator = final_estimator
        self.cv = cv
        self.stack_method = stack_method
        self.n_jobs = n_jobs
        self.passthrough = passthrough
        self.verbose = verbose

    @property
    def named_estimators_(self):
        return {n: e for (n, _), e in zip(self.estimators, self.estimators_)}

    def fit(self, X, y, timer=None, group=None, svc_group=None):
        from .stack_trainer import fit_stacking
        fit_stacking(self, as_tensor(X), as_tensor(y), timer=timer, group=group, svc_group=svc_group)
        return self

    def transform(self, X) -> torch.Tensor:
        cols = [est.predict_proba(X)[:, 1] for est in self.estimators_]
        dev = cols[0].device
        return torch.stack([c.to(dev, torch.float64) for c in cols], dim=1)

    # fused single-kernel inference (ops.stack_infer) for the HF stack on the GPU
    fused_inference = True

    def _packed_stack(self, device):
        key = (id(self.estimators_), id(self.final_estimator_), str(device))
        cached = getattr(self, "_pstack", None)
        if cached is None or cached[0] != key:
            from ..ops.packing import pack_stack
            cached = self._pstack = (key, pack_stack(self, device))
        return cached[1]

    def predict_p1(self, X) -> torch.Tensor:
        """P(class 1) per row.  On the GPU, a fitted HF-shaped stack runs as ONE fused kernel
        (scaler → SVC/Platt, trees, LR → meta LR; f32 output); otherwise per-model."""
        X = as_tensor(X)
        if X.is_cuda and self.fused_inference:
            pk = self._packed_stack(X.device)
            if pk is not None:
                return ops.stack_infer(X, pk)
        return self.final_estimator_.predict_proba(self.transform(X))[:, 1]

    def predict_proba(self, X) -> torch.Tensor:
        X = as_tensor(X)
        if X.is_cuda and self.fused_inference and self._packed_stack(X.device) is not None:
            p1 = self.predict_p1(X).to(torch.float64)
            return torch.stack([1 - p1, p1], dim=1)
        return self.final_estimator_.predict_proba(self.transform(X))

    def decision_function(self, X) -> torch.Tensor:
        return self.final_estimator_.decision_function(self.transform(X))

    def predict(self, X) -> torch.Tensor:
        return (self.predict_proba(X)[:, 1] > 0.5).to(torch.float64)

    def to(self, device):
        for e in self.estimators_:
            e.to(device)
        self.final_estimator_.to(device)
        return self

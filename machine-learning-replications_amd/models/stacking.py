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

    def fit(self, X, y, timer=None, group=None, svc_group=None, plan=None):
        from .stack_trainer import fit_stacking
        fit_stacking(self, as_tensor(X), as_tensor(y), timer=timer, group=group, svc_group=svc_group, plan=plan)
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

    # below this many rows the GPU takes the per-model f64 path: a single patient gets the exact
    # (1e-7 golden) probability, and the fused f32 kernel pays off only on batches
    FUSED_MIN_ROWS = 1024

    # ≤ this many host rows of an HF-shaped stack go through the native f64 host predictor
    # (ops/csrc/host.hip stack_predict_host: single-patient latency, no tensor dispatch)
    HOST_NATIVE_MAX_ROWS = 256

    def _host_pack(self):
        """numpy operands of the native host predictor, or None (not HF-shaped / no extension)."""
        cached = getattr(self, "_hpack", None)
        key = (id(self.estimators_), id(self.final_estimator_))
        if cached is not None and cached[0] == key:
            return cached[1]
        pk = None
        try:
            from .. import ops
            from .gbdt import GradientBoostingClassifier
            from .linear import LogisticRegression
            from .scaler import StandardScaler
            from .svc import SVC
            e = self.estimators_
            # the same shape/flag contract as ops.packing.pack_stack (the fused GPU kernel):
            # no passthrough, an RBF SVC with Platt probabilities, and the scaler's with_mean /
            # with_std flags honoured (identity centre / scale when off)
            if (ops.has_ext() and len(e) == 3 and isinstance(e[0], Pipeline) and len(e[0].steps) == 2
                    and isinstance(e[0].steps[0][1], StandardScaler) and isinstance(e[0].steps[1][1], SVC)
                    and isinstance(e[1], GradientBoostingClassifier) and isinstance(e[2], LogisticRegression)
                    and isinstance(self.final_estimator_, LogisticRegression)
                    and not getattr(self, "passthrough", False)
                    and e[0].steps[1][1].kernel == "rbf" and e[0].steps[1][1].probability
                    and e[0].steps[1][1]._dual_coef_.shape[0] == 1):
                import numpy as np
                sc, svc = e[0].steps[0][1], e[0].steps[1][1]
                g, lr, mt = e[1], e[2], self.final_estimator_
                c = lambda t, dt=np.float64: np.ascontiguousarray(t.detach().cpu().numpy(), dtype=dt)  # noqa: E731
                K = int(g.tree_feature_.shape[1])
                Fs = int(svc.support_vectors_.shape[1])
                mean = c(sc.mean_) if sc.with_mean else np.zeros(Fs)
                scale = c(sc.scale_) if sc.with_std else np.ones(Fs)
                pk = dict(mean=mean, scale=scale, sv=c(svc.support_vectors_),
                          coef=c(svc._dual_coef_[0]), gamma=float(svc._gamma), icpt=float(svc._intercept_[0]),
                          A=float(svc._probA[0]), B=float(svc._probB[0]), T=int(g.tree_feature_.shape[0]), K=K,
                          feat=c(g.tree_feature_, np.int64), thr=c(g.tree_threshold_),
                          left=c(g.tree_left_, np.int64), right=c(g.tree_right_, np.int64),
                          value=c(g.tree_value_.reshape(g.tree_value_.shape[0], -1)[:, :K]),
                          init=float(g.init_raw_), lr=float(g.learning_rate), lrc=c(lr.coef_[0]),
                          lri=float(lr.intercept_[0]), meta=c(mt.coef_[0]), metai=float(mt.intercept_[0]),
                          F=Fs)
                if pk["mean"].size != Fs or pk["scale"].size != Fs or pk["meta"].size != 3 or pk["lrc"].size != pk["F"] or pk["sv"].shape[1] != pk["F"]:
                    pk = None
                else:   # raw pointers resolved once (each .ctypes access costs ~1 µs)
                    pk["args"] = (pk["mean"].ctypes.data, pk["scale"].ctypes.data, pk["sv"].shape[0],
                                  pk["sv"].ctypes.data, pk["coef"].ctypes.data, pk["gamma"], pk["icpt"],
                                  pk["A"], pk["B"], pk["T"], pk["K"], pk["feat"].ctypes.data,
                                  pk["thr"].ctypes.data, pk["left"].ctypes.data, pk["right"].ctypes.data,
                                  pk["value"].ctypes.data, pk["init"], pk["lr"], pk["lrc"].ctypes.data,
                                  pk["lri"], pk["meta"].ctypes.data, pk["metai"])
        except Exception:   # pragma: no cover - any mismatch: the generic per-model path
            pk = None
        self._hpack = (key, pk)
        return pk

    def _host_native_proba(self, X: torch.Tensor):
        """[n, 2] f64 probabilities from the native host predictor, or None."""
        pk = self._host_pack()
        if pk is None or X.dim() != 2 or X.shape[1] != pk["F"]:
            return None
        import numpy as np
        from .. import ops
        x = X.detach().numpy()
        if x.dtype != np.float64 or not x.flags.c_contiguous:
            x = np.ascontiguousarray(x, dtype=np.float64)
        n = x.shape[0]
        out = np.empty((2, n), dtype=np.float64)
        ops.ext().stack_predict_host(n, pk["F"], x.ctypes.data, *pk["args"], out.ctypes.data + 8 * n)
        np.subtract(1.0, out[1], out=out[0])
        return torch.from_numpy(out.T)

    def predict_proba(self, X) -> torch.Tensor:
        X = as_tensor(X)
        if X.shape[0] <= self.HOST_NATIVE_MAX_ROWS:
            # device rows too: one small D2H copy beats a dozen kernel launches, and stays f64
            # (predict_hf.py --device cuda reports the exact golden P)
            pr = self._host_native_proba(X.cpu() if X.is_cuda else X)
            if pr is not None:
                return pr.to(X.device) if X.is_cuda else pr
        if (X.is_cuda and self.fused_inference and X.shape[0] >= self.FUSED_MIN_ROWS
                and self._packed_stack(X.device) is not None):
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

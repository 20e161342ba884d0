"""C-SVC with an RBF kernel and Platt probabilities (reference
``train_ensemble_public.py:44``: ``SVC(class_weight='balanced', probability=True,
random_state=2020)`` behind a ``StandardScaler``).

Semantics follow libsvm as wrapped by sklearn: dual QP with
per-class C (``C·class_weight``), ``gamma='scale'`` = 1/(p·Var(X)), Platt
sigmoid fitted on 5-fold internal cross-validation decision values, and the
iterative pairwise-coupling step even for two classes.  Training runs the
batched GPU SMO solver of :mod:`hfens.models.smo`; many SVC fits (CV folds ×
Platt folds) are solved in one launch.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops
from .base import Estimator, as_tensor, balanced_class_weight


class SVC(Estimator):
    _param_names = ("C", "kernel", "degree", "gamma", "coef0", "shrinking", "probability", "tol",
                    "cache_size", "class_weight", "verbose", "max_iter", "decision_function_shape",
                    "break_ties", "random_state")

    def __init__(self, C=1.0, kernel="rbf", degree=3, gamma="scale", coef0=0.0, shrinking=True,
                 probability=False, tol=1e-3, cache_size=200, class_weight=None, verbose=False,
                 max_iter=-1, decision_function_shape="ovr", break_ties=False, random_state=None):
        if kernel != "rbf":
            raise NotImplementedError("only the RBF kernel of the reference model is supported")
        self.C = C
        self.kernel = kernel
        self.degree = degree
        self.gamma = gamma
        self.coef0 = coef0
        self.shrinking = shrinking
        self.probability = probability
        self.tol = tol
        self.cache_size = cache_size
        self.class_weight = class_weight
        self.verbose = verbose
        self.max_iter = max_iter
        self.decision_function_shape = decision_function_shape
        self.break_ties = break_ties
        self.random_state = random_state

    # ------------------------------------------------------------------ training
    def fit(self, X, y):
        from .smo import fit_svc_batch
        fit_svc_batch([self], [as_tensor(X)], [as_tensor(y)])
        return self

    def resolve_gamma(self, X: torch.Tensor) -> float:
        if self.gamma == "scale":
            v = float(X.to(torch.float64).var(unbiased=False))
            return 1.0 / (X.shape[1] * v) if v != 0 else 1.0
        if self.gamma == "auto":
            return 1.0 / X.shape[1]
        return float(self.gamma)

    def class_weights(self, y: torch.Tensor) -> torch.Tensor:
        if self.class_weight == "balanced":
            return balanced_class_weight(y)
        if self.class_weight is None:
            return torch.ones(2, dtype=torch.float64, device=y.device)
        return torch.tensor([self.class_weight.get(0, 1.0), self.class_weight.get(1, 1.0)],
                            dtype=torch.float64, device=y.device)

    # ------------------------------------------------------------------ inference
    def _libsvm_dec(self, X) -> torch.Tensor:
        X = as_tensor(X, device=self.support_vectors_.device)
        packed = None
        if X.is_cuda:
            packed = getattr(self, "_packed", None)
            if packed is None or packed.svt.device != X.device:
                packed = self._packed = ops.pack_svs(self.support_vectors_, self._dual_coef_[0], X.device)
        return ops.rbf_decision(X, self.support_vectors_, self._dual_coef_[0], self._gamma,
                                self._host_scalars()[0], packed=packed)

    def _host_scalars(self):
        """(libsvm intercept, probA, probB) as host floats — cached by set_fitted, so predicting
        on device tensors costs no device→host reads."""
        hs = getattr(self, "_hs", None)
        if hs is None:
            hs = self._hs = (float(self._intercept_[0]), float(self._probA[0]), float(self._probB[0]))
        return hs

    def decision_function(self, X) -> torch.Tensor:
        # sklearn flips libsvm's sign for the binary case
        return -self._libsvm_dec(X)

    def predict_proba(self, X) -> torch.Tensor:
        if not self.probability:
            raise AttributeError("predict_proba requires probability=True")
        dec = self._libsvm_dec(X)
        _, pa, pb = self._host_scalars()
        p1 = ops.svc_proba1(dec, pa, pb).to(torch.float64)
        return torch.stack([1 - p1, p1], dim=1)

    def predict(self, X) -> torch.Tensor:
        return (self.decision_function(X) > 0).to(torch.float64)

    # ------------------------------------------------------------------ state
    def set_fitted(self, *, support, support_vectors, n_support, dual_coef_libsvm, rho, probA, probB,
                   gamma, class_weight, shape_fit, n_features, device=None):
        """Install a libsvm-convention solution (``dual_coef_libsvm`` = y_i·α_i with
        libsvm's label order, decision = Σ coef·K − rho)."""
        dev = device
        self.n_features_in_ = int(n_features)
        self._gamma = float(gamma)
        self.support_ = as_tensor(support, dev, torch.int32)
        self.support_vectors_ = as_tensor(support_vectors, dev)
        c = as_tensor(dual_coef_libsvm, dev).reshape(1, -1)
        self._dual_coef_ = c
        self.dual_coef_ = -c
        self._hs = (-float(rho), float(probA), float(probB))
        host = [class_weight, n_support, rho, probA, probB]
        if any(isinstance(v, torch.Tensor) and v.device.type != "cpu" for v in host):
            self.class_weight_ = as_tensor(class_weight, dev)
            self._n_support = as_tensor(n_support, dev, torch.int32)
            self._intercept_ = as_tensor([-float(rho)], dev)
            self._probA = as_tensor([probA], dev)
            self._probB = as_tensor([probB], dev)
            self.classes_ = torch.tensor([0, 1], dtype=torch.int64, device=dev)
        else:
            # the host scalars travel in ONE pinned non-blocking copy (six pageable copies were
            # six host-synchronous transfers on the fit's tail)
            cw = np.asarray(class_weight, dtype=np.float64).reshape(-1)
            ns = np.asarray(n_support, dtype=np.float64).reshape(-1)
            small = torch.from_numpy(np.concatenate([cw, [-float(rho), float(probA), float(probB), 0.0, 1.0], ns]))
            if dev is not None and torch.device(dev).type == "cuda":
                small = small.pin_memory().to(dev, non_blocking=True)
            k = cw.shape[0]
            self.class_weight_ = small[:k]
            self._intercept_ = small[k:k + 1]
            self._probA = small[k + 1:k + 2]
            self._probB = small[k + 2:k + 3]
            self.classes_ = small[k + 3:k + 5].to(torch.int64)
            self._n_support = small[k + 5:].to(torch.int32)
        self.intercept_ = -self._intercept_
        self.fit_status_ = 0
        self.shape_fit_ = tuple(int(s) for s in shape_fit)
        self._sparse = False
        self._packed = None
        return self

    def set_platt(self, probA: float, probB: float, dev_pair=None):
        """Install the Platt pair after a :meth:`set_fitted` that ran before the pair was read back
        (the stacking fit's tail: the model's bookkeeping overlaps the Platt kernels).  ``dev_pair``:
        the pair's float64 device copy [A, B] (the Platt kernel's output), used without a copy."""
        self._hs = (self._hs[0], float(probA), float(probB))
        if dev_pair is not None:
            self._probA = dev_pair[0:1]
            self._probB = dev_pair[1:2]
        elif float(probA) != 0.0 or float(probB) != 0.0:
            pair = torch.tensor([float(probA), float(probB)], dtype=torch.float64)
            dev = self._intercept_.device
            if dev.type == "cuda":
                pair = pair.pin_memory().to(dev, non_blocking=True)
            self._probA, self._probB = pair[0:1], pair[1:2]
        return self

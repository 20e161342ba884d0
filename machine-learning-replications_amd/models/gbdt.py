"""Gradient-boosted trees for binary deviance (reference
``train_ensemble_public.py:45``: ``GradientBoostingClassifier(n_estimators=100,
max_depth=1, random_state=2020)``; semantics SURVEY.md E7 / §3.5).

Model layout: every tree is a row of fixed-width node tables ``[T, K]``
(``feature`` < 0 marks a leaf, ``threshold`` float64, ``left``/``right``
children, ``value`` = *unshrunk* Newton leaf value, plus the impurity /
sample-count columns the 0.23.2 checkpoint stores).  Prediction is
``raw = log(p/(1-p))_prior + learning_rate·Σ_t value_t[leaf_t(x)]``.

Training is histogram-based on device (:mod:`hfens.models.hist_gbdt`): features
are quantised to ≤256 bins whose edges are the midpoints of consecutive distinct
values whenever a feature has ≤256 distinct values, so candidate thresholds —
and therefore splits — coincide with sklearn's exact splitter.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import ops
from .base import Estimator, as_tensor

F32_EPS = float(np.finfo(np.float32).eps)


class GradientBoostingClassifier(Estimator):
    _param_names = ("n_estimators", "learning_rate", "loss", "criterion", "min_samples_split",
                    "min_samples_leaf", "min_weight_fraction_leaf", "subsample", "max_features",
                    "max_depth", "min_impurity_decrease", "min_impurity_split", "ccp_alpha", "init",
                    "random_state", "alpha", "verbose", "max_leaf_nodes", "warm_start", "presort",
                    "validation_fraction", "n_iter_no_change", "tol", "max_bins")

    def __init__(self, n_estimators=100, learning_rate=0.1, loss="deviance", criterion="friedman_mse",
                 min_samples_split=2, min_samples_leaf=1, min_weight_fraction_leaf=0.0, subsample=1.0,
                 max_features=None, max_depth=3, min_impurity_decrease=0.0, min_impurity_split=None,
                 ccp_alpha=0.0, init=None, random_state=None, alpha=0.9, verbose=0, max_leaf_nodes=None,
                 warm_start=False, presort="deprecated", validation_fraction=0.1, n_iter_no_change=None,
                 tol=1e-4, max_bins=256):
        self.n_estimators = n_estimators
        self.learning_rate = learning_rate
        self.loss = loss
        self.criterion = criterion
        self.min_samples_split = min_samples_split
        self.min_samples_leaf = min_samples_leaf
        self.min_weight_fraction_leaf = min_weight_fraction_leaf
        self.subsample = subsample
        self.max_features = max_features
        self.max_depth = max_depth
        self.min_impurity_decrease = min_impurity_decrease
        self.min_impurity_split = min_impurity_split
        self.ccp_alpha = ccp_alpha
        self.init = init
        self.random_state = random_state
        self.alpha = alpha
        self.verbose = verbose
        self.max_leaf_nodes = max_leaf_nodes
        self.warm_start = warm_start
        self.presort = presort
        self.validation_fraction = validation_fraction
        self.n_iter_no_change = n_iter_no_change
        self.tol = tol
        self.max_bins = max_bins

    # ------------------------------------------------------------------ training
    def fit(self, X, y, sample_mask=None):
        from .hist_gbdt import fit_gbdt_batch
        X = as_tensor(X)
        y = as_tensor(y, device=X.device)
        masks = None if sample_mask is None else sample_mask[None]
        fit_gbdt_batch([self], X, y, masks)
        return self

    # ------------------------------------------------------------------ inference
    @property
    def init_raw_(self) -> float:
        p1 = float(self.class_prior_[1])
        p1 = min(max(p1, F32_EPS), 1 - F32_EPS)
        return math.log(p1 / (1 - p1))

    def decision_function(self, X) -> torch.Tensor:
        X = as_tensor(X, device=self.tree_value_.device)
        packed = None
        if X.is_cuda:
            packed = getattr(self, "_packed", None)
            if packed is None or packed.nodes.device != X.device:
                packed = self._packed = ops.pack_forest(self.tree_feature_, self.tree_threshold_,
                                                        self.tree_left_, self.tree_right_,
                                                        self.tree_value_, X.device)
        return ops.tree_raw(X, self.tree_feature_, self.tree_threshold_, self.tree_left_,
                            self.tree_right_, self.tree_value_, self.init_raw_,
                            float(self.learning_rate), packed=packed).to(torch.float64)

    def predict_proba(self, X) -> torch.Tensor:
        p1 = torch.sigmoid(self.decision_function(X))
        return torch.stack([1 - p1, p1], dim=1)

    def predict(self, X) -> torch.Tensor:
        return (self.decision_function(X) > 0).to(torch.float64)

    # ------------------------------------------------------------------ state
    def set_fitted(self, *, feature, threshold, left, right, value, impurity, n_node_samples,
                   weighted_n_node_samples, node_count, class_prior, train_score, n_features,
                   rng_state=None, device=None):
        self.n_features_in_ = int(n_features)
        self.n_features_ = int(n_features)
        # (arange: a device fill, not a blocking host→device copy behind the stream's queued work)
        self.classes_ = torch.arange(2, dtype=torch.int64, device=device)
        self.n_classes_ = 2
        self.max_features_ = int(n_features)
        self.tree_feature_ = as_tensor(feature, device, torch.int32)
        self.tree_threshold_ = as_tensor(threshold, device)
        self.tree_left_ = as_tensor(left, device, torch.int32)
        self.tree_right_ = as_tensor(right, device, torch.int32)
        self.tree_value_ = as_tensor(value, device)
        self.tree_impurity_ = as_tensor(impurity, device)
        self.tree_n_node_samples_ = as_tensor(n_node_samples, device, torch.int64)
        self.tree_weighted_n_node_samples_ = as_tensor(weighted_n_node_samples, device)
        self.tree_node_count_ = as_tensor(node_count, device, torch.int32)
        self.class_prior_ = as_tensor(class_prior, device)
        self.train_score_ = as_tensor(train_score, device)
        self.n_estimators_ = int(self.tree_feature_.shape[0])
        self.rng_state_ = rng_state
        self._packed = None
        return self

"""Run configuration.  Defaults reproduce the reference's hard-coded setup
(``train_ensemble_public.py:29-52``; full table SURVEY.md §5.6)."""
from __future__ import annotations

from dataclasses import asdict, dataclass, field
from typing import Optional

import numpy as np


@dataclass
class EnsembleConfig:
    seed: int = 2020                 # init_rs (T:30): SVC / GBC / LassoCV random_state
    lasso_cv: int = 10               # num_xrsval (T:29)
    n_selected: int = 17             # SelectFromModel max_features (T:52)
    knn_neighbors: int = 1           # KNNImputer n_neighbors (T:37)
    svc_C: float = 1.0
    svc_tol: float = 1e-3
    gbc_estimators: int = 100        # T:45
    gbc_depth: int = 1               # T:45
    gbc_learning_rate: float = 0.1
    lr_C: float = 1.0
    meta_C: float = 1.0
    stack_folds: int = 5             # StackingClassifier cv=None → StratifiedKFold(5)
    # 'lg' as the reference gets it: liblinear's default-tolerance iterate, its coordinate order
    # seeded from numpy's global RNG (T:31, T:46; host emulation, models/logreg_solver.py).  False:
    # the device solver's exact optimum (the benchmark's default; the two differ by liblinear's tol)
    liblinear_exact: bool = False

    def to_dict(self):
        return asdict(self)


def build_estimators(cfg: Optional[EnsembleConfig] = None):
    """The reference stack (T:43-48) as native estimators."""
    from .models.gbdt import GradientBoostingClassifier
    from .models.linear import LogisticRegression
    from .models.scaler import StandardScaler
    from .models.stacking import StackingClassifier, make_pipeline
    from .models.svc import SVC
    cfg = cfg or EnsembleConfig()
    estimators = [
        ("svc", make_pipeline(StandardScaler(), SVC(C=cfg.svc_C, tol=cfg.svc_tol, class_weight="balanced",
                                                    probability=True, random_state=cfg.seed))),
        ("gbc", GradientBoostingClassifier(n_estimators=cfg.gbc_estimators, max_depth=cfg.gbc_depth,
                                           learning_rate=cfg.gbc_learning_rate, random_state=cfg.seed)),
        ("lg", LogisticRegression(C=cfg.lr_C, class_weight="balanced", penalty="l1", solver="liblinear")),
    ]
    estimators[2][1].emulate_liblinear = bool(cfg.liblinear_exact)
    return StackingClassifier(estimators=estimators,
                              final_estimator=LogisticRegression(C=cfg.meta_C, class_weight="balanced"))


def build_selector(cfg: Optional[EnsembleConfig] = None):
    from .models.lasso import LassoCV, SelectFromModel
    cfg = cfg or EnsembleConfig()
    return SelectFromModel(LassoCV(random_state=cfg.seed, cv=cfg.lasso_cv), threshold=-np.inf,
                           max_features=cfg.n_selected)

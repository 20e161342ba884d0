"""Common estimator plumbing.

Every estimator keeps its fitted state as torch tensors so a model can live on
an MI355X (``cuda`` device under PyTorch-ROCm) or on the host.  Compute is
routed by the device of the tensors: ``cuda`` tensors go through the
hand-written gfx950 HIP kernels in :mod:`hfens.ops` (which raise if the
extension is missing), host tensors through the plain-PyTorch reference
implementations that the kernel numerics tests compare against.
"""
from __future__ import annotations

import copy
from typing import Any, Dict

import numpy as np
import torch


def as_tensor(x, device=None, dtype=torch.float64) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=device if device is not None else x.device, dtype=dtype)
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device)


class Estimator:
    """Minimal sklearn-like base: hyper-parameters are the ``__init__`` kwargs."""

    _param_names: tuple = ()

    def get_params(self) -> Dict[str, Any]:
        return {k: getattr(self, k) for k in self._param_names}

    def clone(self):
        """Unfitted copy with the same hyper-parameters (sklearn ``clone``).  Immutable parameter
        values (numbers, strings, None) are shared as they are; anything else is deep-copied (the
        stacking trainer clones a dozen estimators per fit on the SVC's critical path)."""
        params = self.get_params()
        if all(v is None or isinstance(v, (bool, int, float, str)) for v in params.values()):
            return type(self)(**params)
        return type(self)(**copy.deepcopy(params))

    def _fitted_tensors(self):
        for k, v in vars(self).items():
            if k.endswith("_") and isinstance(v, torch.Tensor):
                yield k, v

    def to(self, device):
        for k, v in list(self._fitted_tensors()):
            setattr(self, k, v.to(device))
        for v in vars(self).values():
            if isinstance(v, Estimator):
                v.to(device)
            elif isinstance(v, (list, tuple)):
                for e in v:
                    if isinstance(e, Estimator):
                        e.to(device)
                    elif isinstance(e, tuple) and len(e) == 2 and isinstance(e[1], Estimator):
                        e[1].to(device)
        return self

    def __repr__(self):
        args = ", ".join(f"{k}={getattr(self, k)!r}" for k in self._param_names)
        return f"{type(self).__name__}({args})"


def balanced_class_weight(y: torch.Tensor, n_classes: int = 2) -> torch.Tensor:
    """``n_samples / (n_classes * bincount(y))`` (sklearn ``compute_class_weight('balanced')``)."""
    cnt = torch.bincount(y.long(), minlength=n_classes).to(torch.float64)
    return y.numel() / (n_classes * cnt)

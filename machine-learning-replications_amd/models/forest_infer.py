"""Ensemble inference on binned inputs (BASELINE config 5 "deep ensemble").

Histogram-trained trees split on bin boundaries, so an ensemble of depth-1 trees folds exactly
into one lookup table per (model, feature): ``raw_b(x) = init_b + Σ_f T_b[f][bin_f(x)]`` — the
cost per row is F table reads whatever the number of trees (1000 stumps × 5 seeds → 5 × 40
lookups).  ``ops/csrc/forest.hip: binned_stump_raw`` runs it on the GPU; the host path is the
fp64 reference.  Deeper trees use the generic node walk (``ops.tree_raw``).
"""
from __future__ import annotations

from typing import List, Tuple

import torch


def stump_bin_tables(models, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``(T [B, F, 256] f64, init [B] f64)`` for histogram-trained depth-1 GBCs sharing one
    bin mapper."""
    tabs, inits = [], []
    for m in models:
        if getattr(m, "tree_blo_", None) is None or int(m.max_depth) != 1:
            raise ValueError("stump tables need depth-1 trees from the histogram trainer")
        feat = m.tree_feature_[:, 0].to(torch.int64)
        blo = m.tree_blo_[:, 0].to(torch.int64)
        vl = m.tree_value_[:, 1].to(torch.float64)
        vr = m.tree_value_[:, 2].to(torch.float64)
        dev = feat.device if device is None else torch.device(device)
        F = int(m.n_features_in_)
        k = torch.arange(256, device=feat.device)
        split = feat >= 0
        contrib = torch.where(k[None, :] <= blo[:, None], vl[:, None], vr[:, None]) * float(m.learning_rate)
        contrib = contrib * split[:, None]
        T = torch.zeros(F, 256, dtype=torch.float64, device=feat.device)
        T.index_add_(0, feat.clamp(min=0), contrib)
        tabs.append(T.to(dev))
        inits.append(float(m.init_raw_))
    return torch.stack(tabs), torch.tensor(inits, dtype=torch.float64, device=tabs[0].device)


def ensemble_raw_binned(tables: torch.Tensor, init: torch.Tensor, bins: torch.Tensor) -> torch.Tensor:
    """Raw scores ``[B, n]`` of every model for feature-major uint8 ``bins [F, n]``."""
    B, F, _ = tables.shape
    n = bins.shape[1]
    if bins.is_cuda:
        from .. import ops
        t32 = tables.to(device=bins.device, dtype=torch.float32).contiguous()
        ini = init.to(device=bins.device, dtype=torch.float64).contiguous()
        out = torch.empty(B, n, dtype=torch.float32, device=bins.device)
        ops.ext().binned_stump_raw(bins.contiguous().data_ptr(), n, F, t32.data_ptr(), B, ini.data_ptr(),
                                   out.data_ptr(), ops.stream_ptr(bins.device))
        return out
    idx = bins.to(torch.int64)                                   # [F, n]
    g = torch.gather(tables, 2, idx[None].expand(B, F, n))        # [B, F, n]
    return init[:, None] + g.sum(1)

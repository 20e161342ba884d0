"""Feature quantisation for histogram GBDT (SURVEY.md K7 ``quantize_bins``).

Trees compare the float32-cast input (sklearn's tree DTYPE), so bins are built on
``float32(x)``.  A feature with ≤ ``max_bins`` distinct values gets one bin per
distinct value — candidate splits are then exactly sklearn's exact-splitter
candidates and thresholds are midpoints of adjacent present values.  Otherwise
distinct values are grouped into ``max_bins`` quantile groups; a split between
groups uses the midpoint of the left group's max and the right group's min.

With a process group the distinct-value tables are merged across ranks so every
rank bins identically (all-gather of the per-rank value sets).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import torch


@dataclass
class BinMapper:
    nbins: torch.Tensor     # [F] int32
    lo_val: torch.Tensor    # [F, 256] f64 (min value in bin)
    hi_val: torch.Tensor    # [F, 256] f64 (max value in bin)
    uppers: List[torch.Tensor]  # per feature f32 bin upper edges (= hi values)
    max_bins: int

    @property
    def max_nb(self) -> int:
        return int(self.nbins.max())

    def transform(self, X: torch.Tensor) -> torch.Tensor:
        """``X [n, F]`` → feature-major uint8 bins ``[F, n]``."""
        n, F = X.shape
        out = torch.empty(F, n, dtype=torch.uint8, device=X.device)
        X32 = X.to(torch.float32)
        for f in range(F):
            idx = torch.searchsorted(self.uppers[f], X32[:, f].contiguous())
            out[f] = idx.clamp_(max=int(self.nbins[f]) - 1).to(torch.uint8)
        return out


def _distinct(v32: torch.Tensor, group=None):
    u, c = torch.unique(v32, sorted=True, return_counts=True)
    if group is not None:
        from ..parallel import dist as pdist
        u, c = pdist.merge_value_counts(u, c, group)
    return u, c


def fit_bins(X: torch.Tensor, max_bins: int = 256, group=None) -> BinMapper:
    if not 2 <= max_bins <= 256:
        raise ValueError("max_bins must be in [2, 256]")
    n, F = X.shape
    dev = X.device
    X32 = X.to(torch.float32)
    nb = torch.empty(F, dtype=torch.int32)
    lo = torch.zeros(F, 256, dtype=torch.float64)
    hi = torch.zeros(F, 256, dtype=torch.float64)
    uppers = []
    for f in range(F):
        u, c = _distinct(X32[:, f].contiguous(), group)
        u = u.cpu()
        c = c.cpu()
        k = u.numel()
        if k <= max_bins:
            nb[f] = k
            lo[f, :k] = u.double()
            hi[f, :k] = u.double()
            up = u.clone()
        else:
            cum = torch.cumsum(c, 0).double()
            tot = float(cum[-1])
            # group end = last distinct value whose cumulative count reaches the quantile
            targets = torch.arange(1, max_bins, dtype=torch.float64) * (tot / max_bins)
            ends = torch.searchsorted(cum, targets).clamp(max=k - 1)
            ends = torch.unique(torch.cat([ends, torch.tensor([k - 1])]))
            starts = torch.cat([torch.tensor([0]), ends[:-1] + 1])
            g = ends.numel()
            nb[f] = g
            lo[f, :g] = u[starts].double()
            hi[f, :g] = u[ends].double()
            up = u[ends].clone()
        uppers.append(up.to(dev, torch.float32).contiguous())
    return BinMapper(nb.to(dev), lo.to(dev), hi.to(dev), uppers, max_bins)

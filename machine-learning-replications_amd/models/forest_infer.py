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


# ============================================================================ fp8 leaf values
# BASELINE config 5 ("deep ensemble, fp8 leaf values on CDNA4 MFMA"): the ensemble as a leaf
# one-hot × leaf-value GEMV on the matrix cores (ops/csrc/forest_fp8.hip).  Leaf values are
# stored as OCP fp8 e4m3 in two terms per model (hi = fp8(σv), lo = fp8(σv − hi), σ a per-model
# power of two); the MFMA's 16 output columns hold [hi_0..hi_{S−1} | lo_0..lo_{S−1}].
_E4M3_TOP = 224.0   # largest |σ·v| target: room for the hi term's rounding below e4m3's 448


class Fp8Forest:
    """Packed fp8 leaf-value GEMV operands for ≤ 8 histogram-trained GBCs of equal depth/trees."""

    def __init__(self, models, device=None):
        m0 = models[0]
        S = len(models)
        if not 1 <= S <= 8:
            raise ValueError("Fp8Forest packs 1..8 models (hi/lo columns of one 16-wide MFMA tile)")
        if any(getattr(m, "tree_blo_", None) is None for m in models):
            raise ValueError("fp8 forest needs histogram-trained trees (split bins)")
        d = int(m0.max_depth)
        T = int(m0.n_estimators_)
        if any(int(m.max_depth) != d or int(m.n_estimators_) != T for m in models):
            raise ValueError("models must share depth and tree count")
        dev = torch.device(device) if device is not None else m0.tree_feature_.device
        L = 1 << d
        NI = L - 1
        K = T * L
        self.d, self.T, self.S, self.L = d, T, S, L
        self.F = int(m0.n_features_in_)
        # tree table (shared layout, per model): [S][T][NI] u16 = (blo << 8) | feat, 255 = leaf
        nodes = torch.empty(S, T, NI, dtype=torch.int32)
        V = torch.zeros(S, K, dtype=torch.float64)
        for s, m in enumerate(models):
            feat = m.tree_feature_[:, :NI].to(torch.int64).cpu()
            blo = m.tree_blo_[:, :NI].to(torch.int64).cpu()
            leafnode = feat < 0
            nodes[s] = torch.where(leafnode, torch.full_like(feat, 255), feat | (blo << 8)).to(torch.int32)
            val = m.tree_value_.to(torch.float64).cpu() * float(m.learning_rate)
            # virtual path v (bit lev = MSB-first decision) → the leaf value the walk reaches; under an
            # early leaf the device always goes left, every virtual slot below it gets that value
            for v in range(L):
                h = torch.zeros(T, dtype=torch.int64)
                done = torch.zeros(T, dtype=torch.bool)
                for lev in range(d):
                    bit = (v >> (d - 1 - lev)) & 1
                    isleaf = m.tree_feature_.cpu().gather(1, h[:, None])[:, 0] < 0
                    done |= isleaf
                    h = torch.where(done, h, 2 * h + 1 + bit)
                V[s, torch.arange(T) * L + v] = val.gather(1, h[:, None])[:, 0]
        # all models' trees concatenated (tree s·T + t): the one-hot over K = S·T·L slots is shared,
        # V is block-diagonal — model s's slots carry values in columns s (hi) and S + s (lo) only
        self._nodes_i32 = nodes
        self.V64 = V
        vmax = V.abs().amax(1).clamp(min=1e-300)
        sigma = torch.exp2(torch.floor(torch.log2(_E4M3_TOP / vmax)))
        Vs = (V * sigma[:, None]).to(torch.float32)
        hi = Vs.to(torch.float8_e4m3fn)
        lo = (Vs - hi.to(torch.float32)).to(torch.float8_e4m3fn)
        self.hi, self.lo = hi, lo
        self.inv_scale = (1.0 / sigma).to(torch.float32)
        self.init = torch.tensor([float(m.init_raw_) for m in models], dtype=torch.float64)
        Kall = S * K
        # K steps of 128 slots (gfx950 v_mfma_scale_f32_16x16x128_f8f6f4): lane ℓ = 16·g + column
        # holds slots 128q + 32g + j, j < 32, of its column — the A side's order (forest_fp8.hip)
        self.Q = Q = -(-Kall // 128)
        Bm = torch.zeros(Q * 128, 16, dtype=torch.uint8)
        for s_ in range(S):
            Bm[s_ * K:(s_ + 1) * K, s_] = hi[s_].view(torch.uint8)
            Bm[s_ * K:(s_ + 1) * K, S + s_] = lo[s_].view(torch.uint8)
        frag = Bm.view(Q, 4, 32, 16).permute(0, 1, 3, 2).reshape(Q, 64, 32).contiguous()   # [q][lane][j]
        self.bfrag = frag.view(torch.int64).reshape(Q * 64 * 4)
        self.nodes_all = nodes.reshape(S * T, NI).to(torch.int16)   # (blo << 8 | feat) ≤ 0xFFFF as i16 bits
        self.device = dev
        self._dev_cache = None

    def _operands(self, device):
        if self._dev_cache is None or self._dev_cache[0] != device:
            self._dev_cache = (device, self.nodes_all.to(device), self.bfrag.to(device),
                               self.inv_scale.to(device), self.init.to(device))
        return self._dev_cache[1:]

    def raw(self, bins: torch.Tensor) -> torch.Tensor:
        """Raw scores [S, n] for feature-major uint8 bins [F, n] (the models' shared bin mapper)."""
        F, n = bins.shape
        if not bins.is_cuda:
            return self.reference_raw(bins)
        from .. import ops
        nodes, bfrag, inv_scale, init = self._operands(bins.device)
        out = torch.empty(self.S, n, dtype=torch.float32, device=bins.device)
        b = bins.contiguous()
        ops.ext().forest_fp8(b.data_ptr(), n, n, F, self.S * self.T, self.d, nodes.data_ptr(), bfrag.data_ptr(),
                             self.Q, self.S, inv_scale.data_ptr(), init.data_ptr(), out.data_ptr(),
                             ops.stream_ptr(bins.device))
        return out

    def reference_raw(self, bins: torch.Tensor, exact: bool = False) -> torch.Tensor:
        """fp64 PyTorch reference of the SAME quantised operands (walk, gather hi + lo); ``exact``:
        the unquantised f64 leaf values instead (the binned model the fp8 GEMV approximates).

        Binned inference equals the threshold walk on new rows wherever the split threshold is a
        global bin edge — always for depth-1 trees on all rows; a deeper node whose rows leave a
        bin empty puts sklearn's threshold at the node-local midpoint, and an unseen value inside
        that gap may take the other side here."""
        b = bins.to(torch.int64).cpu()
        n = b.shape[1]
        out = torch.empty(self.S, n, dtype=torch.float64)
        for s in range(self.S):
            nd = self._nodes_i32[s]                      # [T, NI]
            h = torch.zeros(self.T, n, dtype=torch.int64)
            for _ in range(self.d):
                code = nd.gather(1, h)                   # [T, n]
                f = code & 0xFF
                blo = code >> 8
                fb = b[f.clamp(max=b.shape[0] - 1), torch.arange(n)[None, :].expand(self.T, n)]
                right = (f != 255) & (fb > blo)
                h = 2 * h + 1 + right.to(torch.int64)
            leaf = h - (self.L - 1)
            slot = torch.arange(self.T)[:, None] * self.L + leaf
            if exact:
                out[s] = self.init[s] + self.V64[s][slot].sum(0)
            else:
                v = self.hi[s].to(torch.float64)[slot] + self.lo[s].to(torch.float64)[slot]
                out[s] = self.init[s] + v.sum(0) * float(self.inv_scale[s])
        return out.to(bins.device)

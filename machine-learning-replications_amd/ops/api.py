"""Op entry points: validate, then route ``cuda`` tensors to the HIP extension and
host tensors to :mod:`hfens.ops.reference`."""
from __future__ import annotations

import torch

from . import reference as ref
from .packing import pack_forest, pack_stack, pack_svs

__all__ = ["rbf_decision", "svc_proba1", "tree_raw", "expit", "pack_svs", "pack_forest", "pack_stack",
           "stack_infer", "weighted_moments"]


def _c(t: torch.Tensor, dtype) -> torch.Tensor:
    return t.to(dtype).contiguous()


def rbf_decision(z, sv, coef, gamma: float, intercept: float, packed=None):
    """libsvm RBF decision values; ``packed`` = cached :class:`PackedSV` for ``sv``/``coef``."""
    if z.is_cuda:
        from . import ext, stream_ptr
        pk = packed if packed is not None else pack_svs(sv, coef, z.device)
        z32 = _c(z, torch.float32)
        n, F = z32.shape
        if F != pk.F:
            raise ValueError(f"rbf_decision: X has {F} features, model has {pk.F}")
        out = torch.empty(n, dtype=torch.float32, device=z.device)
        ext().rbf_decision(z32.data_ptr(), n, F, pk.svt.data_ptr(), pk.sn.data_ptr(), pk.coef.data_ptr(),
                           pk.mp, float(gamma), float(intercept), out.data_ptr(), stream_ptr(z.device))
        return out
    return ref.rbf_decision(z, sv, coef, gamma, intercept)


def svc_proba1(dec, A: float, B: float):
    if dec.is_cuda:
        from . import ext, stream_ptr
        d32 = _c(dec, torch.float32)
        out = torch.empty_like(d32)
        ext().svc_proba1(d32.data_ptr(), out.data_ptr(), d32.numel(), float(A), float(B),
                         stream_ptr(dec.device))
        return out
    return ref.svc_proba1(dec, A, B)


def tree_raw(x, feature, threshold, left, right, value, init: float, lr: float, packed=None):
    if x.is_cuda:
        from . import ext, stream_ptr
        pk = packed if packed is not None else pack_forest(feature, threshold, left, right, value, x.device)
        x32 = _c(x, torch.float32)
        n, F = x32.shape
        if pk.max_feature >= F:
            raise ValueError("tree_raw: a split feature index exceeds the input width")
        out = torch.empty(n, dtype=torch.float32, device=x.device)
        ext().forest_raw(x32.data_ptr(), n, F, pk.nodes.data_ptr(), pk.values.data_ptr(), pk.n_trees,
                         pk.max_nodes, float(init), float(lr), out.data_ptr(), stream_ptr(x.device))
        return out
    return ref.tree_raw(x, feature, threshold, left, right, value, init, lr)


def stack_infer(x, pk, out=None, grid: int = 0, stream=None):
    """Fused P(class 1) of the whole HF stack (one kernel, one pass over ``x``).
    ``x``: [n, F] f32 or f64; ``pk``: :class:`PackedStack` on ``x``'s device.  Returns f32 on
    the GPU (written into ``out`` if given), f64 on the host."""
    if x.is_cuda:
        from . import ext, stream_ptr
        if x.dtype not in (torch.float32, torch.float64):
            x = x.to(torch.float32)
        x = x.contiguous()
        n, F = x.shape
        if F != pk.F:
            raise ValueError(f"stack_infer: X has {F} features, model has {pk.F}")
        if out is None:
            out = torch.empty(n, dtype=torch.float32, device=x.device)
        elif out.dtype != torch.float32 or out.numel() < n or not out.is_contiguous():
            raise ValueError("stack_infer: out must be a contiguous f32 buffer of >= n elements")
        f, s, st = pk.forest, pk.sv, pk.stumps
        ext().stack_infer(x.data_ptr(), int(x.dtype == torch.float64), n, F, s.mp, f.n_trees, f.max_nodes,
                          -pk.gamma * 1.4426950408889634, pk.svc_b, pk.probA, pk.probB, pk.gb_init,
                          pk.gb_lr, pk.lr_b, pk.meta_w[0], pk.meta_w[1], pk.meta_w[2], pk.meta_b,
                          pk.mean.data_ptr(), pk.inv_scale.data_ptr(), s.svt.data_ptr(), s.sn.data_ptr(),
                          s.coef.data_ptr(), f.nodes.data_ptr(), f.values.data_ptr(), pk.lr_w.data_ptr(),
                          st.off.data_ptr() if st is not None else 0,
                          st.pairs.data_ptr() if st is not None else 0,
                          st.base if st is not None else 0.0,
                          out.data_ptr(), int(grid),
                          stream if stream is not None else stream_ptr(x.device))
        return out[:n]
    return ref.stack_infer(x, pk)


def expit(x):
    return torch.sigmoid(x)


def weighted_moments(X, W, V=None):
    """``G[p] = Σ_n W[p,n] x_n x_nᵀ``, ``a[p] = Σ_n W[p,n] x_n``, ``v[p] = Σ_n V[p,n] x_n`` (f64)."""
    X = X.to(torch.float64).contiguous()
    W = W.to(torch.float64).contiguous()
    n, F = X.shape
    P = W.shape[0]
    if X.is_cuda:
        from . import ext, stream_ptr
        C = (n + 127) // 128
        npairs = F * (F + 1) // 2
        Gp = torch.empty(P, C, npairs, dtype=torch.float64, device=X.device)
        ap = torch.empty(P, C, F, dtype=torch.float64, device=X.device)
        vp = torch.empty(P, C, F, dtype=torch.float64, device=X.device)
        Vc = V.to(torch.float64).contiguous() if V is not None else None
        ext().weighted_moments(X.data_ptr(), n, F, W.data_ptr(), Vc.data_ptr() if Vc is not None else 0,
                               P, Gp.data_ptr(), ap.data_ptr(), vp.data_ptr(), stream_ptr(X.device))
        Gu = Gp.sum(1)
        iu = torch.triu_indices(F, F, device=X.device)
        G = torch.zeros(P, F, F, dtype=torch.float64, device=X.device)
        G[:, iu[0], iu[1]] = Gu
        G[:, iu[1], iu[0]] = Gu
        return G, ap.sum(1), (vp.sum(1) if V is not None else None)
    G = torch.einsum("pn,ni,nj->pij", W, X, X)
    a = W @ X
    v = V.to(torch.float64) @ X if V is not None else None
    return G, a, v

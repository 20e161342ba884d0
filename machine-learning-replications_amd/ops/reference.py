"""Plain-PyTorch reference implementations of every device op.

These define the semantics the gfx950 HIP kernels must reproduce and run the
host (CPU) path.  They follow the algorithms the reference delegates to
(libsvm / sklearn trees / liblinear), re-derived from the published math; see
the per-function notes and SURVEY.md §2.2 (E2-E12).
"""
from __future__ import annotations

import math

import torch

LOG2E = 1.4426950408889634


# ----------------------------------------------------------------------------- SVC inference
def rbf_decision(z: torch.Tensor, sv: torch.Tensor, coef: torch.Tensor, gamma: float,
                 intercept: float, chunk: int = 65536) -> torch.Tensor:
    """``dec_i = Σ_j coef_j · exp(-γ‖z_i − sv_j‖²) + intercept`` (libsvm ``svm_predict_values``,
    RBF kernel ``k(x,y)=exp(-γ‖x−y‖²)``)."""
    out = torch.empty(z.shape[0], dtype=z.dtype, device=z.device)
    for s in range(0, z.shape[0], chunk):
        zz = z[s:s + chunk]
        d2 = ((zz[:, None, :] - sv[None, :, :]) ** 2).sum(-1)
        out[s:s + chunk] = torch.exp(-gamma * d2) @ coef + intercept
    return out


def sigmoid_predict(dec: torch.Tensor, A: float, B: float) -> torch.Tensor:
    """Platt ``1/(1+exp(A·f+B))`` evaluated in libsvm's overflow-safe form."""
    fApB = dec * A + B
    pos = torch.exp(-fApB.clamp(min=0)) / (1.0 + torch.exp(-fApB.clamp(min=0)))
    neg = 1.0 / (1.0 + torch.exp(fApB.clamp(max=0)))
    return torch.where(fApB >= 0, pos, neg)


def couple2(r01: torch.Tensor, max_iter: int = 100) -> torch.Tensor:
    """Two-class pairwise coupling (Wu, Lin & Weng 2004, method 2 — the iterative
    solver libsvm's ``multiclass_probability`` runs even for k = 2), vectorised over
    rows.  Input r01 = P(class 0 | {0,1}); returns p1 = P(class 1).  Stopping rule
    ``max_t |(Qp)_t − pᵀQp| < 0.005/k``."""
    r10 = 1.0 - r01
    q00 = r10 * r10
    q11 = r01 * r01
    q01 = -r10 * r01
    p0 = torch.full_like(r01, 0.5)
    p1 = torch.full_like(r01, 0.5)
    eps = 0.005 / 2
    active = torch.ones_like(r01, dtype=torch.bool)
    for _ in range(max_iter):
        qp0 = q00 * p0 + q01 * p1
        qp1 = q01 * p0 + q11 * p1
        pqp = p0 * qp0 + p1 * qp1
        err = torch.maximum((qp0 - pqp).abs(), (qp1 - pqp).abs())
        active = active & ~(err < eps)
        if not bool(active.any()):
            break
        # t = 0 update
        d = (-qp0 + pqp) / q00
        np0 = p0 + d
        npqp = (pqp + d * (d * q00 + 2 * qp0)) / (1 + d) / (1 + d)
        nqp0 = (qp0 + d * q00) / (1 + d)
        nqp1 = (qp1 + d * q01) / (1 + d)
        np0 = np0 / (1 + d)
        np1 = p1 / (1 + d)
        # t = 1 update
        d = (-nqp1 + npqp) / q11
        np1 = np1 + d
        np0 = np0 / (1 + d)
        np1 = np1 / (1 + d)
        p0 = torch.where(active, np0, p0)
        p1 = torch.where(active, np1, p1)
    return p1


def svc_proba1(dec: torch.Tensor, A: float, B: float) -> torch.Tensor:
    """libsvm ``svm_predict_probability`` for two classes → P(class 1)."""
    r01 = sigmoid_predict(dec, A, B).clamp(1e-7, 1 - 1e-7)
    return couple2(r01)


# ----------------------------------------------------------------------------- tree inference
def tree_raw(x: torch.Tensor, feature: torch.Tensor, threshold: torch.Tensor, left: torch.Tensor,
             right: torch.Tensor, value: torch.Tensor, init: float, lr: float) -> torch.Tensor:
    """Sum of tree outputs ``init + lr·Σ_t value_t[leaf_t(x)]``.  Decision rule
    ``float32(x[f]) <= threshold`` → left (sklearn compares the float32-cast input
    against the float64 threshold).  Arrays are [T, K] node tables, leaves have
    feature < 0."""
    x32 = x.to(torch.float32).to(torch.float64)
    n = x.shape[0]
    T = feature.shape[0]
    # all trees walk together ([T, n] node ids, one step per level: a handful of tensor ops
    # instead of ~10 per tree), then the per-tree contributions are added in tree order
    # (cumsum over [init, lr·v_0, …] reproduces sklearn's sequential raw += lr·v_t rounding)
    node = torch.zeros(T, n, dtype=torch.long, device=x.device)
    cols = torch.arange(n, device=x.device)[None, :].expand(T, n)
    feature = feature.long()
    for _ in range(feature.shape[1]):
        f = feature.gather(1, node)
        leaf = f < 0
        if bool(leaf.all()):
            break
        fv = x32[cols, f.clamp(min=0)]
        go_left = fv <= threshold.gather(1, node)
        nxt = torch.where(go_left, left.long().gather(1, node), right.long().gather(1, node))
        node = torch.where(leaf, node, nxt)
    v = value.to(torch.float64).reshape(T, -1).gather(1, node)          # [T, n]
    terms = torch.cat([torch.full((1, n), float(init), dtype=torch.float64, device=x.device), lr * v])
    return torch.cumsum(terms, 0)[-1]


def expit(x: torch.Tensor) -> torch.Tensor:
    return torch.sigmoid(x)


# ----------------------------------------------------------------------------- fused stack
def stack_infer(x: torch.Tensor, pk) -> torch.Tensor:
    """fp64 reference of the fused ``stack_infer`` kernel on a :class:`PackedStack` (host
    tensors): scaler → RBF SVC (Platt + coupling) / trees / L1-LR → meta LR, P(class 1)."""
    x = x.to(torch.float64)
    F = pk.F
    z = (x - pk.mean.to(torch.float64)) * pk.inv_scale.to(torch.float64)
    sv = pk.sv.svt[:F].t().to(torch.float64)
    dec = rbf_decision(z, sv, pk.sv.coef.to(torch.float64), pk.gamma, pk.svc_b)
    p_svc = svc_proba1(dec, pk.probA, pk.probB)
    if pk.stumps is not None:
        st = pk.stumps
        x32 = x.to(torch.float32).to(torch.float64)
        raw = torch.full((x.shape[0],), st.base, dtype=torch.float64)
        off = st.off.tolist()
        for f in range(F):
            for j in range(off[f], off[f + 1]):
                t, d = float(st.pairs[j, 0]), float(st.pairs[j, 1])
                raw += (x32[:, f] > t).to(torch.float64) * d
    else:
        nd = pk.forest.nodes.reshape(pk.forest.n_trees, pk.forest.max_nodes, 4)
        thr = nd[..., 3].contiguous().view(torch.float32).to(torch.float64)
        raw = tree_raw(x, nd[..., 0], thr, nd[..., 1], nd[..., 2],
                       pk.forest.values.reshape(pk.forest.n_trees, -1), pk.gb_init, pk.gb_lr)
    p_gbc = torch.sigmoid(raw)
    p_lg = torch.sigmoid(x @ pk.lr_w.to(torch.float64) + pk.lr_b)
    w0, w1, w2 = pk.meta_w
    return torch.sigmoid(pk.meta_b + w0 * p_svc + w1 * p_gbc + w2 * p_lg)

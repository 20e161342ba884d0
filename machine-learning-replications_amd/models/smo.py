"""Batched C-SVC training with libsvm semantics.

Licence: the host mirrors ``_smo_host`` / ``_sigmoid_train_host`` follow LIBSVM
(BSD-3-Clause, Chang & Lin; THIRD_PARTY_NOTICES.md).

``fit_svc_batch`` trains any number of RBF ``SVC(probability=True)`` fits at once.
Each fit expands into libsvm's problems:

* Platt CV (``svm_binary_svc_probability``): the class-grouped training set is
  shuffled with libsvm's RNG (``std::mt19937`` seeded with sklearn's
  ``RandomState(random_state).randint(INT_MAX)``, Lemire-bounded draws), split into
  5 contiguous folds; each fold's training part is a sub-problem whose points are
  re-grouped by sorted label (class 1 first) with per-class C;
* the final solve on the class-grouped problem (class 0 = internal +1).

All problems of all fits get their RBF Gram matrix from one batched MFMA launch
(``gram_rbf_batch``) and are solved by one batched SMO launch (``smo_batch``, one
workgroup per problem).  Held-out Platt decision values use the MFMA
``rbf_decision`` kernel and the sigmoids are fitted by ``platt_batch``.  The host
path mirrors every step in numpy (used on CPU and by the kernel tests).
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from ..utils.hostread import landed, stage   # early read-backs polled on their data

TAU = 1e-12
INT_MAX = np.iinfo(np.int32).max


# ----------------------------------------------------------------------------- libsvm RNG
class _MTStream:
    """Raw std::mt19937 output (numpy's legacy int seeding == init_genrand)."""

    def __init__(self, seed: int):
        self._bg = np.random.RandomState(seed & 0xFFFFFFFF)._bit_generator
        self._buf = np.empty(0, dtype=np.uint64)
        self._pos = 0

    def next(self) -> int:
        if self._pos >= self._buf.size:
            self._buf = self._bg.random_raw(4096)
            self._pos = 0
        v = int(self._buf[self._pos])
        self._pos += 1
        return v


def bounded_rand_int(mt: _MTStream, rng: int) -> int:
    """sklearn newrand.h ``bounded_rand_int`` (tweaked Lemire)."""
    x = mt.next()
    m = x * rng
    lo = m & 0xFFFFFFFF
    if lo < rng:
        t = (-rng) & 0xFFFFFFFF
        if t >= rng:
            t -= rng
            if t >= rng:
                t %= rng
        while lo < t:
            x = mt.next()
            m = x * rng
            lo = m & 0xFFFFFFFF
    return m >> 32


def libsvm_perm(l: int, seed: int) -> np.ndarray:
    from .. import ops
    if ops.has_ext():  # native host loop (ops/csrc/host.hip)
        out = np.empty(l, dtype=np.int64)
        ops.ext().libsvm_perm(l, int(seed) & 0xFFFFFFFF, out.ctypes.data)
        return out
    return libsvm_perm_py(l, seed)


def libsvm_perm_py(l: int, seed: int) -> np.ndarray:
    mt = _MTStream(seed)
    perm = np.arange(l)
    for i in range(l):
        j = i + bounded_rand_int(mt, l - i)
        perm[i], perm[j] = perm[j], perm[i]
    return perm


_SEED_CACHE: dict = {}


def sklearn_libsvm_seed(random_state) -> int:
    """``check_random_state(random_state).randint(np.iinfo('i').max)`` (sklearn svm/_base.py).
    An int seed always gives the same draw: cached (a RandomState construction costs ~0.2 ms)."""
    if isinstance(random_state, (int, np.integer)) and not isinstance(random_state, bool):
        k = int(random_state)
        if k not in _SEED_CACHE:
            _SEED_CACHE[k] = int(np.random.RandomState(k).randint(INT_MAX))
        return _SEED_CACHE[k]
    if random_state is None:
        rs = np.random.mtrand._rand
    elif isinstance(random_state, (int, np.integer)):
        rs = np.random.RandomState(int(random_state))
    else:
        rs = random_state
    return int(rs.randint(INT_MAX))


# ----------------------------------------------------------------------------- problems
@dataclass
class _Prob:
    fit: int
    fold: int             # -1 = final solve
    rows: Optional[np.ndarray]   # int64 indices into the fit's Z, in problem order (None: constant fold)
    npos: int
    Cp: float
    Cn: float
    gamma: float
    held: Optional[np.ndarray] = None       # Platt: held-out grouped positions
    held_rows: Optional[np.ndarray] = None  # … and their rows of Z
    const: float = 0.0
    colmap: Optional[np.ndarray] = None     # Platt sub-problem: column map into its fit's final Gram (planned ahead)

    @property
    def l(self) -> int:
        return 0 if self.rows is None else int(self.rows.shape[0])


def _expand(fit_id, y_np: np.ndarray, gamma: float, cw: np.ndarray, svc):
    """libsvm problem list of one SVC fit — pure host index bookkeeping on the labels, so preparing
    the 36 problems costs no device round trips (native: ops/csrc/host.hip svc_expand_host, one call;
    :func:`_expand_py` is the numpy original, equal array for array — tests/test_smo_host.py)."""
    from .. import ops
    if NATIVE_EXPAND and ops.has_ext():
        return _expand_native(fit_id, y_np, gamma, cw, svc)
    return _expand_py(fit_id, y_np, gamma, cw, svc)


NATIVE_EXPAND = os.environ.get("HFENS_NATIVE_EXPAND", "1") != "0"


def _expand_native(fit_id, y_np: np.ndarray, gamma: float, cw: np.ndarray, svc):
    from .. import ops
    y = np.ascontiguousarray(y_np, dtype=np.float64)
    l = int(y.shape[0])
    seed = sklearn_libsvm_seed(svc.random_state) & 0xFFFFFFFF if svc.probability else -1
    out = np.empty((7 if svc.probability else 1) * l, dtype=np.int64)
    meta = np.empty(21, dtype=np.int64)
    ops.ext().svc_expand_host(y.ctypes.data, l, seed, out.ctypes.data, meta.ctypes.data)
    return _wrap_expansion(fit_id, l, out, meta, gamma, cw, svc)


def _wrap_expansion(fit_id, l: int, out: np.ndarray, meta: np.ndarray, gamma, cw, svc):
    """The problem list of one fit from the native expansion's arrays (svc_expand_host layout)."""
    grouped = out[:l]
    n0 = int(meta[0])
    C0, C1 = float(svc.C * cw[0]), float(svc.C * cw[1])
    probs = []
    if svc.probability:
        perm, gp, rows_all = out[l:2 * l], out[2 * l:3 * l], out[3 * l:]
        for k in range(5):
            b, e = k * l // 5, (k + 1) * l // 5
            n1, nn0, off, ln = (int(v) for v in meta[1 + 4 * k:5 + 4 * k])
            held = perm[b:e]
            if n1 == 0 or nn0 == 0:
                probs.append(_Prob(fit_id, k, None, 0, 0.0, 0.0, gamma, held, gp[b:e],
                                   const=1.0 if n1 == 0 else -1.0))
                continue
            probs.append(_Prob(fit_id, k, rows_all[off:off + ln], n1, C1, C0, gamma, held, gp[b:e]))
    probs.append(_Prob(fit_id, -1, grouped, n0, C0, C1, gamma))
    return probs, dict(grouped=grouped, n0=n0, l=l, gamma=gamma, C0=C0, C1=C1)


def _expand_py(fit_id, y_np: np.ndarray, gamma: float, cw: np.ndarray, svc):
    yb = y_np > 0.5
    idx0 = np.nonzero(~yb)[0]
    idx1 = np.nonzero(yb)[0]
    grouped = np.concatenate([idx0, idx1]).astype(np.int64)
    n0, l = int(idx0.shape[0]), int(grouped.shape[0])
    C0, C1 = float(svc.C * cw[0]), float(svc.C * cw[1])
    probs = []
    if svc.probability:
        seed = sklearn_libsvm_seed(svc.random_state)
        perm = libsvm_perm(l, seed)
        gp = grouped[perm]                     # rows in permutation order
        cls0_at = perm < n0                    # grouped position < n0 ⇔ class 0
        i1, i0 = np.nonzero(~cls0_at)[0], np.nonzero(cls0_at)[0]   # perm positions per class
        g1, g0 = gp[i1], gp[i0]
        for k in range(5):
            b, e = k * l // 5, (k + 1) * l // 5
            # training rows = perm minus [b, e), in perm order, class 1 (label −1) first
            lo1, hi1 = np.searchsorted(i1, (b, e))
            lo0, hi0 = np.searchsorted(i0, (b, e))
            n1 = int(lo1 + i1.shape[0] - hi1)
            nn0 = int(lo0 + i0.shape[0] - hi0)
            held = perm[b:e]
            if n1 == 0 or nn0 == 0:
                probs.append(_Prob(fit_id, k, None, 0, 0.0, 0.0, gamma, held, gp[b:e],
                                   const=1.0 if n1 == 0 else -1.0))
                continue
            rows = np.concatenate([g1[:lo1], g1[hi1:], g0[:lo0], g0[hi0:]])
            probs.append(_Prob(fit_id, k, rows, n1, C1, C0, gamma, held, gp[b:e]))
    probs.append(_Prob(fit_id, -1, grouped, n0, C0, C1, gamma))
    return probs, dict(grouped=grouped, n0=n0, l=l, gamma=gamma, C0=C0, C1=C1)


def plan_svc_problems(svc, y_fits) -> Optional[list]:
    """The label-only half of :func:`launch_svc_batch`, computable before the fit's inputs exist:
    every fit's libsvm problem expansion (γ filled in at launch) and, for each Platt sub-problem,
    the column map into its fit's final-problem Gram (:func:`_column_map`).  ``None`` when the labels
    are not 0/1 (the launch then reads them from the device as usual)."""
    pre = []
    for f, yh in enumerate(y_fits):
        y_np = np.asarray(yh, dtype=np.float64).reshape(-1)
        if not ((y_np == 0.0) | (y_np == 1.0)).all():
            return None
        probs, mt = _expand(f, y_np, None, _class_weights_host(svc, y_np), svc)
        final = probs[-1]
        # (the column maps serve the stored-Gram exact solver only; the working-set solver, which
        # takes every batch from WS_MIN_POINTS points on, never reads them)
        if final.l <= _MAP_MAX and (SOLVER == "exact" or (SOLVER == "auto" and final.l < WS_MIN_POINTS)):
            inv = np.full(int(final.rows.max()) + 1, -1, dtype=np.int64)
            inv[final.rows] = np.arange(final.l)
            for p in probs[:-1]:
                if p.rows is not None and p.l <= _MAP_MAX:
                    p.colmap = _column_map(final, p, inv)
        pre.append((y_np, probs, mt))
    return pre


def _class_weights_host(svc, y_np: np.ndarray) -> np.ndarray:
    if svc.class_weight == "balanced":
        cnt = np.bincount((y_np > 0.5).astype(np.int64), minlength=2).astype(np.float64)
        return y_np.shape[0] / (2 * cnt)
    return svc.class_weights(torch.as_tensor(y_np)).cpu().numpy()


def _to_dev(a: np.ndarray, device) -> torch.Tensor:
    """Host index array → device without blocking the host (pinned, non-blocking)."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    if torch.device(device).type != "cuda":
        return t
    return t.pin_memory().to(device, non_blocking=True)


def _gather_rows(Zs, probs, attr, device) -> torch.Tensor:
    """Concatenate Zs[p.fit][getattr(p, attr)] over ``probs`` with one gather per fit — or ONE
    gather when every Zs[f] is a row block of one matrix (the stacking trainer's batched scaler
    output: one upload and two launches instead of six of each)."""
    fits = sorted({p.fit for p in probs})
    base = Zs[0]._base
    if (base is not None and base.dim() == 2 and base.is_contiguous() and base.storage_offset() == 0
            and all(Z._base is base and Z.is_contiguous() for Z in Zs)):
        F = base.shape[1]
        order, idx, offs = [], [], []
        for f in fits:
            sub = [p for p in probs if p.fit == f]
            off = Zs[f].storage_offset() // F
            for p in sub:
                idx.append(getattr(p, attr))
                offs.append(off)
            order += sub
        if [id(p) for p in order] != [id(p) for p in probs]:
            raise AssertionError("problems must be grouped by fit")
        # the global row indices written straight into pinned memory (one pass, no staging copy)
        total = sum(int(a.shape[0]) for a in idx)
        cuda = torch.device(device).type == "cuda"
        h = torch.empty(total, dtype=torch.int64, pin_memory=cuda)
        cat = h.numpy()
        pos = 0
        for a, off in zip(idx, offs):
            np.add(a, off, out=cat[pos:pos + a.shape[0]], casting="unsafe")
            pos += a.shape[0]
        ii = h.to(device, non_blocking=True) if cuda else h
        return base.index_select(0, ii).to(torch.float32)
    parts = []
    order = []
    for f in fits:
        idx = [getattr(p, attr) for p in probs if p.fit == f]
        if not idx:
            continue
        ii = _to_dev(np.concatenate(idx), device)
        parts.append(Zs[f].index_select(0, ii).to(torch.float32))
        order += [p for p in probs if p.fit == f]
    if [id(p) for p in order] != [id(p) for p in probs]:
        raise AssertionError("problems must be grouped by fit")
    return torch.cat(parts).contiguous()


# ----------------------------------------------------------------------------- host solver
def _smo_host(K: np.ndarray, npos: int, Cp: float, Cn: float, eps: float, max_iter: int):
    l = K.shape[0]
    pos = np.arange(l) < npos
    C = np.where(pos, Cp, Cn)
    G = -np.ones(l)
    alpha = np.zeros(l)
    st = np.zeros(l, dtype=np.int8)
    it = 0
    for it in range(max_iter):
        up = np.where(pos, st != 2, st != 0)
        if not up.any():
            break
        v = np.where(up, np.where(pos, -G, G), -np.inf)
        Gmax = v.max()
        i = int(np.flatnonzero(v == Gmax)[-1])
        yi = 1 if pos[i] else -1
        Ki = K[i].astype(np.float64)
        low = np.where(pos, st != 0, st != 2)
        yG = np.where(pos, G, -G)
        gmax2 = yG[low].max() if low.any() else -np.inf
        gd = Gmax + yG
        cand = low & (gd > 0)
        quad = 2.0 - 2.0 * Ki
        quad[quad <= 0] = TAU
        nobj = np.where(cand, gd * gd / quad, -np.inf)
        if not cand.any() or Gmax + gmax2 < eps:
            break
        best = nobj.max()
        j = int(np.flatnonzero(nobj == best)[-1])
        yj = 1 if pos[j] else -1
        Ci, Cj = C[i], C[j]
        Qij = yi * yj * float(K[i, j])
        ai, aj = alpha[i], alpha[j]
        Gi, Gj = G[i], G[j]
        ai_old, aj_old = ai, aj
        if yi != yj:
            qc = 2.0 + 2.0 * Qij
            qc = qc if qc > 0 else TAU
            delta = (-Gi - Gj) / qc
            diff = ai - aj
            ai += delta
            aj += delta
            if diff > 0:
                if aj < 0:
                    aj, ai = 0.0, diff
            else:
                if ai < 0:
                    ai, aj = 0.0, -diff
            if diff > Ci - Cj:
                if ai > Ci:
                    ai, aj = Ci, Ci - diff
            else:
                if aj > Cj:
                    aj, ai = Cj, Cj + diff
        else:
            qc = 2.0 - 2.0 * Qij
            qc = qc if qc > 0 else TAU
            delta = (Gi - Gj) / qc
            s = ai + aj
            ai -= delta
            aj += delta
            if s > Ci:
                if ai > Ci:
                    ai, aj = Ci, s - Ci
            else:
                if aj < 0:
                    aj, ai = 0.0, s
            if s > Cj:
                if aj > Cj:
                    aj, ai = Cj, s - Cj
            else:
                if ai < 0:
                    ai, aj = 0.0, s
        dai, daj = ai - ai_old, aj - aj_old
        yv = np.where(pos, 1.0, -1.0)
        G += yv * (yi * Ki * dai + yj * K[j].astype(np.float64) * daj)
        alpha[i], alpha[j] = ai, aj
        st[i] = 2 if ai >= Ci else (0 if ai <= 0 else 1)
        st[j] = 2 if aj >= Cj else (0 if aj <= 0 else 1)
    yG = np.where(pos, G, -G)
    free = st == 1
    if free.any():
        rho = yG[free].sum() / free.sum()
    else:
        ubm = np.where(pos, st == 0, st == 2)
        lbm = np.where(pos, st == 2, st == 0)
        ub = yG[ubm].min() if ubm.any() else np.inf
        lb = yG[lbm].max() if lbm.any() else -np.inf
        rho = (ub + lb) / 2
    return alpha, float(rho), it


def _gram_host(Zp: np.ndarray, gamma: float) -> np.ndarray:
    sq = (Zp * Zp).sum(1)
    d2 = np.maximum(sq[:, None] + sq[None, :] - 2.0 * Zp @ Zp.T, 0.0)
    K = np.exp(-gamma * d2).astype(np.float32)
    np.fill_diagonal(K, 1.0)
    return K


def _sigmoid_train_host(dec, labels):
    prior1 = float((labels > 0).sum())
    prior0 = float(labels.size - prior1)
    hiT, loT = (prior1 + 1.0) / (prior1 + 2.0), 1 / (prior0 + 2.0)
    t = np.where(labels > 0, hiT, loT)
    A, B = 0.0, np.log((prior0 + 1.0) / (prior1 + 1.0))

    def f(a, b):
        fApB = dec * a + b
        return np.where(fApB >= 0, t * fApB + np.log1p(np.exp(-np.abs(fApB))),
                        (t - 1) * fApB + np.log1p(np.exp(-np.abs(fApB)))).sum()
    fval = f(A, B)
    for _ in range(100):
        fApB = dec * A + B
        p = np.where(fApB >= 0, np.exp(-fApB) / (1 + np.exp(-fApB)), 1 / (1 + np.exp(fApB)))
        q = 1 - p
        d2 = p * q
        h11 = (dec * dec * d2).sum() + 1e-12
        h22 = d2.sum() + 1e-12
        h21 = (dec * d2).sum()
        d1 = t - p
        g1, g2 = (dec * d1).sum(), d1.sum()
        if abs(g1) < 1e-5 and abs(g2) < 1e-5:
            break
        det = h11 * h22 - h21 * h21
        dA = -(h22 * g1 - h21 * g2) / det
        dB = -(-h21 * g1 + h11 * g2) / det
        gd = g1 * dA + g2 * dB
        step = 1.0
        while step >= 1e-10:
            nA, nB = A + step * dA, B + step * dB
            nf = f(nA, nB)
            if nf < fval + 0.0001 * step * gd:
                A, B, fval = nA, nB, nf
                break
            step /= 2.0
        if step < 1e-10:
            break
    return A, B


# ----------------------------------------------------------------------------- device helpers
_GRAM_DT = np.dtype([("zoff", "<i8"), ("koff", "<i8"), ("l", "<i4"), ("ld", "<i4"), ("ngl2e", "<f4"),
                     ("pad", "<i4")])
_SMO_DT = np.dtype([("koff", "<i8"), ("aoff", "<i8"), ("l", "<i4"), ("ld", "<i4"), ("npos", "<i4"),
                    ("pad", "<i4"), ("Cp", "<f8"), ("Cn", "<f8")])
_PLATT_DT = np.dtype([("off", "<i8"), ("l", "<i4"), ("n0", "<i4")])
_DEC_DT = np.dtype([("zoff", "<i8"), ("hoff", "<i8"), ("l", "<i4"), ("h", "<i4"), ("ngl2e", "<f4"),
                    ("per", "<i4")])


def _dev_struct(arr: np.ndarray, device) -> torch.Tensor:
    """Small descriptor table → device without blocking the host: a pageable H2D copy is
    host-synchronous and waits for everything queued before it on the stream (e.g. the SMO
    launch), which would serialise the caller's overlap with other streams."""
    host = torch.from_numpy(arr.view(np.uint8).copy())
    if torch.device(device).type != "cuda":
        return host
    return host.pin_memory().to(device, non_blocking=True)


_WS_DT = np.dtype([("zoff", "<i8"), ("aoff", "<i8"), ("l", "<i4"), ("npos", "<i4"), ("Cp", "<f8"),
                   ("Cn", "<f8"), ("ngl2e", "<f4"), ("pad", "<i4")])
_WS_STATE_BYTES = 88     # sizeof(WsState) in svm_ws.hip


WS_MAX_F = 48            # features the working-set kernel's register/LDS budget admits


# K-cached rounds (svm_ws.hip ws_kc_round_kernel): q = 256 with the working set's kernel matrix in
# LDS and a one-wave pair loop; for F ≤ WS_KC_MAX_F.  HFENS_SVM_WS_KC=0 keeps the q = 1024 solver.
# "auto": K-cached rounds for problems past the one-workgroup selector (> WS_KC_DIRECT_MAX points,
# candidate-list selection), the q = 1024 solver below that: on the bench's 10k problem the K-cached
# rounds measured 44 vs 33 ms per fit (226 rounds of ≈ 45 µs selection + build against 35 of the
# q = 1024 solver, profiles/r4_headline.md).  "1": always (F ≤ 24); "0": never.
WS_KC = os.environ.get("HFENS_SVM_WS_KC", "auto")
WS_KC_MAX_F = 24
WS_KC_Q = 256
WS_KC_DIRECT_MAX = 16 * 1024      # svm_ws.hip kWsDirectMax: larger problems select from candidate lists


def ws_kc(F: int, max_l: int = 0) -> bool:
    if WS_KC == "0" or F > WS_KC_MAX_F:
        return False
    return WS_KC == "1" or max_l > WS_KC_DIRECT_MAX


# working-set size of the recomputing solver for F ≤ 24 (512: half the slots per pair, more rounds)
WS_Q = int(os.environ.get("HFENS_SVM_WS_Q", "1024"))


def ws_q(F: int, max_l: int = 0) -> int:
    """Working-set size of svm_ws.hip for F features (K-cached: 256; else one slot per thread with
    z_B in LDS: 1024 / 512)."""
    if ws_kc(F, max_l):
        return WS_KC_Q
    return WS_Q if (F <= 24 and WS_Q in (512, 1024)) else 1024 if F <= 24 else 512


def _ws_ks(F: int) -> int:
    ks = (F + 1) // 2
    return 4 if ks <= 4 else 9 if ks <= 9 else 12 if ks <= 12 else 24

# Device solver: "exact" = libsvm's pair sequence on a stored Gram (svm.hip / svm_coop.hip), "ws" =
# working-set decomposition (svm_ws.hip: q = 1024 slots solved inside one CU with the RBF recomputed
# in registers, half of each working set reused, MFMA gradient updates; O(n) memory).  On the
# bench's 10k problem the exact sequence is ~7.6k pairs at ~7.7 µs (cross-CU hand-offs), the
# working-set solver ~35 rounds of ~250 in-CU pairs (scripts/ws_sim.py).  "auto": ws from
# WS_MIN_POINTS points on (the exact sequence stays for small problems, where it is cheap and
# libsvm-identical), exact when F exceeds the working-set kernel's register budget.
SOLVER = os.environ.get("HFENS_SVM_SOLVER", "auto")
WS_MIN_POINTS = int(os.environ.get("HFENS_SVM_WS_MIN", "4096"))


def _pick_solver(max_l: int, F: int = 17) -> str:
    if SOLVER in ("exact", "ws"):
        return SOLVER
    return "ws" if (max_l >= WS_MIN_POINTS and F <= WS_MAX_F) else "exact"


# Cooperative exact SMO (ops/csrc/svm_coop.hip): every problem's points are split over W
# workgroups that exchange their WSS partials inside the launch — the same pair sequence as the
# one-workgroup smo_kernel, with 1/W of each Gram row read per CU.  A pair is latency-bound either
# way (profiles/r1_smo_latency.md): the one-workgroup kernel waits on two 40 KB row reads through
# one CU, the members on two in-launch exchanges (≈2 µs each); W = 4 measured best on the bench
# (87 vs 95 ms/step with one workgroup), more members add exchange skew.  W ≤ COOP_MAX_W, one
# member per CU, COOP_RESERVE_CUS CUs left to the GBC/LR kernels of the concurrent stream, and
# ≥ COOP_MIN_SLICE points per member.
COOP = os.environ.get("HFENS_SMO_COOP", "1") != "0"
COOP_MIN_SLICE = int(os.environ.get("HFENS_SMO_COOP_SLICE", "384"))
COOP_RESERVE_CUS = int(os.environ.get("HFENS_SMO_COOP_RESERVE", "60"))   # CUs left to concurrent GBC/LR
# more members: exchange skew outweighs the split.  Measured on the bench (36 problems, max l 10k,
# L2 row prefetch on, scripts/probes/gpu_coop_sweep.sh): W=2 89.4, 3 85.0, 4 81.8-85.3, 5 79.8-80.9,
# 6 84.9, 7 125.6 ms/fit (7 leaves 4 CUs to GBC/LR)
_COOP_MAX_W = int(os.environ.get("HFENS_SMO_COOP_MAXW", "5"))
_COOP_GRANULES = 2 * 16 * 10          # exchange slots per problem: 2 × kMaxMembers × kGran (u64)
# "otf" (HFENS_SMO_OTF=1, while a member's rows fit its registers: ≤ 1024 points per member, ≤ 20
# features): the cooperative kernel recomputes its Gram-row entries per pair with the Gram kernel's
# exact expression instead of reading a stored Gram — no O(l²) matrix, no Gram launch, no HBM reads
# per pair, the same pair sequence (tested).  Its exchanges carry the rows (28 granules per member
# instead of 10), which cost more than the row reads they replace at the member counts that fit.
COOP_OTF = os.environ.get("HFENS_SMO_OTF", "0") == "1"   # measured slower than the stored Gram at 4-16 members
_OTF_MAX_S, _OTF_MAX_F = 1024, 20   # ≤ 2 points per thread: no register spill (measured)
_OTF_GRANULES = 2 * 16 * 32          # exchange slots per problem: 2 × kMaxMembers × kOtfGran (u64)
_OTF_DT = np.dtype([("zoff", "<i8"), ("aoff", "<i8"), ("l", "<i4"), ("npos", "<i4"), ("S", "<i4"),
                    ("ngl2e", "<f4"), ("Cp", "<f8"), ("Cn", "<f8")])
_COOP_DT = np.dtype([("koff", "<i8"), ("aoff", "<i8"), ("moff", "<i8"), ("l", "<i4"), ("ld", "<i4"),
                     ("npos", "<i4"), ("S", "<i4"), ("lphys", "<i4"), ("pad", "<i4"), ("Cp", "<f8"), ("Cn", "<f8")])
# Platt-CV sub-problems read their fit's final-problem Gram through a column map (svm_coop.hip
# smo_coop_kernel<K4, Mapped>): a sub-problem's rows are a subset of the same scaled rows with the
# same γ, so its Gram is a principal submatrix of the parent's, entry for entry.  Only the 6 final
# problems' Grams are computed (bench: 1.7 instead of 7 GB written); cooperative solver only.
SHARE_GRAM = os.environ.get("HFENS_SMO_SHARE_GRAM", "1") != "0"
_MAP_MAX = 1 << 15   # column / index keys are packed into 15 bits each
_NCU: dict = {}
# set while re-solving a batch whose cooperative launch reported a member-exchange timeout: the
# one-workgroup solver needs no co-residency (same pair sequence, so the same result)
_FORCE_SINGLE = [False]


def _num_cus(device) -> int:
    d = torch.device(device)
    if d not in _NCU:
        _NCU[d] = int(torch.cuda.get_device_properties(d).multi_processor_count)
    return _NCU[d]


def coop_members(P: int, max_l: int, ncu: int, resident: int = None) -> int:
    """Workgroups per problem for the cooperative SMO (1 = the one-workgroup kernel).

    Co-residency by construction: P·W members must all be resident at once,
    so W is bounded by what the device co-schedules of the kernel (``resident``: occupancy per CU
    × CUs, :func:`coop_resident`; one member per CU at most) minus the COOP_RESERVE_CUS left to
    the concurrent GBC/LR stream.  A member that still arrives late (other work holding its CU)
    costs at most one exchange deadline (HFENS_SMO_WAIT_MS, 20 ms; svm_coop.hip) before the
    whole launch gives up and the batch is re-solved by the one-workgroup kernel."""
    if not COOP or PROFILE_SMO or P <= 0 or _FORCE_SINGLE[0]:
        return 1
    cap = min(ncu, resident if resident is not None else ncu) - COOP_RESERVE_CUS
    if cap < 2 * P:
        return 1
    return max(1, min(_COOP_MAX_W, cap // P, -(-max_l // COOP_MIN_SLICE)))


_RESIDENT: dict = {}


def coop_resident(device) -> int:
    """Blocks of the cooperative kernel the device co-schedules (hipOccupancy… × CUs)."""
    d = torch.device(device)
    if d not in _RESIDENT:
        from .. import ops
        out = np.zeros(2, dtype=np.int64)
        with torch.cuda.device(d):
            ops.ext().coop_resident_blocks(out.ctypes.data)
        _RESIDENT[d] = int(out[0])
    return _RESIDENT[d]


def _gram_parents(live) -> List[int]:
    """For every problem, the index in ``live`` of the problem whose stored Gram it reads (−1: its
    own): a Platt sub-problem (fold ≥ 0) reads its fit's final problem's, when that one is in the
    same launch and both fit the 15-bit keys."""
    final = {p.fit: k for k, p in enumerate(live) if p.fold < 0}
    out = []
    for p in live:
        q = final.get(p.fit, -1) if p.fold >= 0 else -1
        if q >= 0 and (live[q].l > _MAP_MAX or p.l > _MAP_MAX):
            q = -1
        out.append(q)
    return out


def _column_map(par: _Prob, sub: _Prob, inv: Optional[np.ndarray] = None) -> np.ndarray:
    """int32 [par.l]: the sub-problem's index of each parent column (−1: not in the sub-problem).
    ``inv``: the parent's row → column inverse, when already built (shared by its sub-problems)."""
    if inv is None:
        inv = np.full(int(par.rows.max()) + 1, -1, dtype=np.int64)
        inv[par.rows] = np.arange(par.l)
    cols = inv[sub.rows]
    if (cols < 0).any():
        raise AssertionError("Platt sub-problem rows must be rows of the final problem")
    m = np.full(par.l, -1, dtype=np.int32)
    m[cols] = np.arange(sub.l, dtype=np.int32)
    return m


def _solve_exact(E, live, zcat, zoffs, aoffs, F, device, eps, max_iter_cap, s):
    max_l = max(p.l for p in live)
    max_iter = max(10_000_000, 100 * max_l) if max_iter_cap is None else max_iter_cap
    W = coop_members(len(live), max_l, _num_cus(device), coop_resident(device))
    if W > 1 and COOP_OTF and not PROFILE_COOP and F <= _OTF_MAX_F and -(-max_l // W) <= _OTF_MAX_S:
        op = np.zeros(len(live), _OTF_DT)
        for k, p in enumerate(live):
            op[k] = (zoffs[k], aoffs[k], p.l, p.npos, -(-p.l // W), -p.gamma * 1.4426950408889634, p.Cp, p.Cn)
        odev = _dev_struct(op, device)
        alpha = torch.empty(aoffs[-1], dtype=torch.float64, device=device)
        rho = torch.empty(len(live), dtype=torch.float64, device=device)
        iters = torch.empty(len(live), dtype=torch.int32, device=device)
        gap = torch.empty(len(live), dtype=torch.float64, device=device)
        xchg = torch.empty(len(live) * _OTF_GRANULES, dtype=torch.int64, device=device)
        err = torch.zeros(1, dtype=torch.int32, device=device)
        E.smo_coop_otf_batch(odev.data_ptr(), len(live), W, F, int(op["S"].max()), zcat.data_ptr(),
                             alpha.data_ptr(), xchg.data_ptr(), eps, max_iter, rho.data_ptr(), iters.data_ptr(),
                             gap.data_ptr(), err.data_ptr(), s)
        LAST_SMO_INFO.update(members=W, problems=len(live), max_l=max_l, solver="coop-otf")
        return alpha, rho, iters, err
    W = coop_members(len(live), max_l, _num_cus(device), coop_resident(device))
    parent = _gram_parents(live) if (W > 1 and SHARE_GRAM) else [-1] * len(live)
    own = [k for k in range(len(live)) if parent[k] < 0]
    g = np.zeros(len(own), _GRAM_DT)
    sm = np.zeros(len(live), _SMO_DT)
    koff = 0
    for r, k in enumerate(own):
        p = live[k]
        l = p.l
        ld = (l + 63) // 64 * 64
        g[r] = (zoffs[k], koff, l, ld, -p.gamma * 1.4426950408889634, 0)
        sm[k] = (koff, aoffs[k], l, ld, p.npos, 0, p.Cp, p.Cn)
        koff += l * ld
    for k, q in enumerate(parent):
        if q >= 0:
            sm[k] = (sm[q]["koff"], aoffs[k], live[k].l, sm[q]["ld"], live[k].npos, 0, live[k].Cp, live[k].Cn)
    max_own = max(live[k].l for k in own)
    from .. import runtime
    K = runtime.workspace(device, "svm_gram", koff, torch.float32)   # process-lifetime, grown only
    gdev = _dev_struct(g, device)
    E.gram_rbf_batch(zcat.data_ptr(), F, gdev.data_ptr(), len(own), max_own, K.data_ptr(), s)
    from ..utils.timing import hmark
    hmark("svc_gram_launched")
    alpha = torch.empty(aoffs[-1], dtype=torch.float64, device=device)
    rho = torch.empty(len(live), dtype=torch.float64, device=device)
    iters = torch.empty(len(live), dtype=torch.int32, device=device)
    gap = torch.empty(len(live), dtype=torch.float64, device=device)
    max_iter = max(10_000_000, 100 * max_l) if max_iter_cap is None else max_iter_cap
    err = None
    if W > 1:
        cp = np.zeros(len(live), _COOP_DT)
        maps, moff = [], 0
        for k, p in enumerate(live):
            q = parent[k]
            lphys = p.l if q < 0 else live[q].l
            S = -(-(-(-lphys // W)) // 4) * 4
            m = -1
            if q >= 0:
                m = moff
                cm = getattr(p, "colmap", None)
                maps.append(cm if cm is not None and cm.shape[0] == lphys else _column_map(live[q], p))
                moff += lphys
            cp[k] = (sm[k]["koff"], aoffs[k], m, p.l, sm[k]["ld"], p.npos, S, lphys, 0, p.Cp, p.Cn)
        cdev = _dev_struct(cp, device)
        mdev = _to_dev(np.concatenate(maps), device) if maps else None
        xchg = torch.empty(len(live) * _COOP_GRANULES, dtype=torch.int64, device=device)
        err = torch.zeros(1, dtype=torch.int32, device=device)
        prof = torch.zeros(len(live) * 7, dtype=torch.int64, device=device) if PROFILE_COOP else None
        E.smo_coop_batch(cdev.data_ptr(), len(live), W, int(cp["S"].max()), K.data_ptr(),
                         mdev.data_ptr() if mdev is not None else 0, alpha.data_ptr(), xchg.data_ptr(), eps,
                         max_iter, rho.data_ptr(), iters.data_ptr(), gap.data_ptr(), err.data_ptr(),
                         prof.data_ptr() if prof is not None else 0, s)
        if prof is not None:
            LAST_SMO_PROF.update(phases=prof.view(-1, 7).cpu().numpy(), iters=iters.cpu().numpy(),
                                 l=np.array([p.l for p in live]),
                                 names=["step2", "red2", "xchg2", "pair", "update", "red1", "xchg1"])
    else:
        sdev = _dev_struct(sm, device)
        prof = torch.zeros(len(live) * 5, dtype=torch.int64, device=device) if PROFILE_SMO else None
        E.smo_batch(sdev.data_ptr(), len(live), max_l, K.data_ptr(), alpha.data_ptr(), eps, max_iter,
                    rho.data_ptr(), iters.data_ptr(), gap.data_ptr(), prof.data_ptr() if prof is not None else 0, s)
        if prof is not None:
            LAST_SMO_PROF.update(phases=prof.view(-1, 5).cpu().numpy(), iters=iters.cpu().numpy(),
                                 l=np.array([p.l for p in live]))
    LAST_SMO_INFO.update(members=W, problems=len(live), max_l=max_l, solver="coop" if W > 1 else "single",
                         grams=len(own))
    del K
    return alpha, rho, iters, err


# inner stop: local gap < frac·gap0.  Swept on the headline (profiles/r3_runs/ws_sweep, 10 steps each):
# 0.05 39.1, 0.1 34.3, 0.15 33.7, 0.2 31.4-31.8, 0.25 32.2, 0.3 32.8 ms/fit — 0.2 moves 13 % fewer pairs
# (8.6k vs 9.9k on the critical problem) in about as many rounds (35 vs 34)
WS_INNER_FRAC = float(os.environ.get("HFENS_SVM_WS_FRAC", "0.2"))
# the same for the group holding the largest problem (the fit's critical path when groups run
# side by side); host simulation of the bench's 10k problem (scripts/probes/ws_qsim.py, q = 1024):
# 0.2 → 37 rounds / 8.4k pairs, 0.3 → 39 / 8.0k, 0.4 → 46 / 7.9k
WS_INNER_FRAC_BIG = float(os.environ.get("HFENS_SVM_WS_FRAC_BIG", str(WS_INNER_FRAC)))
# inner pairs per round: the 36 problems advance in lock-step rounds, so one long inner solve holds
# up every other problem's next round; a cap bounds that wait (the capped problem simply continues
# in its next working set)
WS_MAX_INNER = int(os.environ.get("HFENS_SVM_WS_INNER", "4096"))
WS_ROUNDS_AHEAD = int(os.environ.get("HFENS_SVM_WS_AHEAD", "64"))      # rounds enqueued without a host check
# … for a cascade-seeded batch, per 10k points of its largest problem (scaled up above 10k): the
# bench's seeded problems need ≤ 24 rounds, and every round past a problem's convergence is three
# no-op launches its group's stream still runs before the finish — measured (profiles/r6_runs/r6av,
# traced medians on one box): SMO done 15.2–15.4 ms at 48 rounds ahead, 14.8 at 32, 14.7 at 28.  A
# batch that needs more rounds reports err and is re-solved with host-checked rounds (correct,
# slower: tests/test_svm_ws_gpu.py)
WS_SEEDED_AHEAD = int(os.environ.get("HFENS_SVM_WS_SEEDED_AHEAD", "32"))
# the K-cached solver's rounds are ~4× as many (q = 256): on the bench's 10k-point problem ≈ 190
WS_KC_ROUNDS_AHEAD = int(os.environ.get("HFENS_SVM_WS_KC_AHEAD", "288"))
# HIP-graph replay of the rounds: "1" K-cached rounds only, "all" the q = 1024 rounds too, "0" off.
# ("all" re-measured in round 6, when the prelaunched stack's host enqueue — 38 ws_steps calls,
# ≈ 450 kernel launches, 1.7 ms of host time per fit — sat on the critical path: no gain, 19.2 /
# 20.4 vs 19.3 / 18.9 ms, profiles/r6_runs/r6g; ROCm's graph launch costs about as much host time
# per node as a direct launch)
WS_GRAPH = os.environ.get("HFENS_SVM_WS_GRAPH", "1")
WS_GRAPH_CHUNK = int(os.environ.get("HFENS_SVM_WS_GRAPH_CHUNK", "32"))   # rounds per captured graph
_WS_GRAPHS: dict = {}
WS_BIG_CHUNK = int(os.environ.get("HFENS_SVM_WS_BIG_CHUNK", "64"))
WS_THREADS = int(os.environ.get("HFENS_SVM_WS_THREADS", "256"))      # inner-solver workgroup (256 or 512)
WS_G0_FIRST = os.environ.get("HFENS_SVM_WS_G0_FIRST", "1") == "1"
# the last (smallest-problem) group on a side stream of its own (runtime FIT_STREAMS svc_ws_2, normal
# priority) instead of the caller's high-priority stream
WS_LAST_SIDE = os.environ.get("HFENS_SVM_WS_LAST_SIDE", "0") == "1"
_WS_SYNC = [False]   # set while re-solving a batch that did not converge within WS_ROUNDS_AHEAD


# Lock-step decoupling: one round kernel ends when its SLOWEST problem's inner solve does, so the
# largest problems (the final fits, l = n) wait every round on the CV folds' solves and vice versa
# (measured on the bench: 22 ms of rounds for a 17.5 ms critical problem).  Problems are grouped by
# size class (a class: l within WS_SPLIT_FRAC of its largest member), at most WS_GROUPS groups (the
# smallest classes share the last); every group runs its rounds on a stream of its own and is
# lock-step only within itself.  WS_GROUPS = 1: one group.
WS_SPLIT_FRAC = float(os.environ.get("HFENS_SVM_WS_SPLIT", "0.95"))
WS_GROUPS = int(os.environ.get("HFENS_SVM_WS_GROUPS", "3"))
WS_EVENTS = os.environ.get("HFENS_WS_EVENTS", "0") == "1"
LAST_WS_EVENTS: dict = {}
_WS_ENQ_CHUNK = int(os.environ.get("HFENS_SVM_WS_ENQ_CHUNK", "4"))   # rounds per group per host enqueue turn


def _ws_groups(live, device) -> List[List[int]]:
    P = len(live)
    if (WS_GROUPS <= 1 or P < 2 or torch.device(device).type != "cuda"
            or not torch.cuda.is_available()):
        return [list(range(P))]
    order = sorted(range(P), key=lambda k: (-live[k].l, k))
    groups: List[List[int]] = []
    for k in order:
        if groups and (live[k].l >= WS_SPLIT_FRAC * live[groups[-1][0]].l or len(groups) == WS_GROUPS):
            groups[-1].append(k)
        else:
            groups.append([k])
    return [sorted(g) for g in groups]


def _solve_ws(E, live, zcat, zoffs, aoffs, F, device, eps, max_iter_cap, s, steps_per_check=None,
              seed=None, q=None, groups=None, deps_out=None, after_first=None):
    """``seed``: a feasible α (per point, this batch's layout) to start from instead of α = 0
    (:func:`_cascade_seed`) — every value AT a bound or at least f32 resolution inside it (the
    selection keys read f64 α, the inner solve f32 α: a value within an f32 ulp of a bound is free
    to one and bound to the other, profiles/r6_nystrom_seed.md); ``q``: the working-set size (default :func:`ws_q`); ``after_first``:
    host work (no device dependency on the rounds) run once every group's first rounds are
    enqueued."""
    P = len(live)
    n = aoffs[-1]
    ml = _max_l(live)
    kc_all = ws_kc(F, ml)          # one solver kind for the whole batch (every group)
    Q = ws_q(F, ml) if (q is None or kc_all) else int(q)
    Fp2 = 2 * _ws_ks(F)
    max_outer = (max(5_000, ml // 4) if max_iter_cap is None else int(max_iter_cap))
    max_inner = WS_MAX_INNER
    # large problems (candidate-list selection, hundreds to thousands of rounds): host-checked rounds
    # in chunks of WS_BIG_CHUNK from the start, one group (the rounds-ahead guess would be far off)
    big = kc_all and ml > WS_KC_DIRECT_MAX
    sync = _WS_SYNC[0] or big
    if big and steps_per_check is None:
        steps_per_check = WS_BIG_CHUNK
    groups = (_ws_groups(live, device) if groups is None else [list(range(P))]) if not sync else [list(range(P))]
    cuda = torch.device(device).type == "cuda"
    caller = torch.cuda.current_stream(device) if cuda else None
    # HIP graphs of the rounds (K-cached, rounds enqueued ahead): ~290 rounds × 2 launches × 3 groups
    # per fit cost as much host time as the device spends on them, so each group's rounds are
    # captured once (WS_GRAPH_CHUNK rounds per graph) and replayed.  Every argument of a captured
    # launch must be the same buffer at every replay: the per-point arrays, the features and every
    # per-group buffer are process-lifetime workspaces (runtime.workspace), re-filled per fit.
    use_graph = (WS_GRAPH != "0" and cuda and (kc_all or WS_GRAPH == "all") and not sync and not PROFILE_WS
                 and caller.cuda_stream != torch.cuda.default_stream(device).cuda_stream)
    # per-point arrays (indexed by each problem's absolute offset) are shared by the groups
    if use_graph:
        from .. import runtime
        zc = runtime.workspace(device, "ws_zcat", zcat.numel(), torch.float32)
        zc.copy_(zcat.reshape(-1))
        zcat = zc
        zn = runtime.workspace(device, "ws_zn", n, torch.float32)
        alpha = runtime.workspace(device, "ws_alpha", n, torch.float64)
        G = runtime.workspace(device, "ws_G", n, torch.float64)
        keys = runtime.workspace(device, "ws_keys", 2 * n, torch.int32)
        hist = runtime.workspace(device, "ws_hist", 1, torch.int32)
    else:
        zn = torch.empty(n, dtype=torch.float32, device=device)
        alpha = torch.empty(n, dtype=torch.float64, device=device)
        G = torch.empty(n, dtype=torch.float64, device=device)
        keys = torch.zeros(2 * n, dtype=torch.int32, device=device)
        hist = torch.zeros(1, dtype=torch.int32, device=device)   # (unused slot kept in the ABI)
    runs = []
    ahead = (WS_KC_ROUNDS_AHEAD if kc_all else
             (-(-WS_SEEDED_AHEAD * max(ml, 10000) // 10000) if seed is not None else WS_ROUNDS_AHEAD))
    left = min(ahead, max_outer)
    chunk = WS_GRAPH_CHUNK if use_graph else _WS_ENQ_CHUNK
    done = [0] * len(groups)
    # the first group (the largest problems: the batch's critical path) gets its first rounds
    # enqueued as soon as its own state is, before the other groups' states are built
    g0_first = WS_G0_FIRST and not sync and not use_graph and len(groups) > 1
    for gi, idx in enumerate(groups):
        # the last (smallest) group on the caller's stream, the others on process-lifetime side streams
        side = None
        if gi == len(groups) - 1 and not (WS_LAST_SIDE and cuda and gi > 0):
            st = s
        else:
            from .. import runtime
            side = runtime.stream(device, f"svc_ws_{gi}", priority=-1)
            side.wait_stream(caller)
            st = side.cuda_stream
        runs.append(_ws_group(E, live, idx, zcat, zoffs, aoffs, F, device, eps, max_outer, max_inner, st,
                              side, zn, alpha, G, keys, hist, n, Q, Fp2, kc_all, gi=gi if use_graph else None,
                              cap_stream=(side if side is not None else caller) if use_graph else None,
                              frac=WS_INNER_FRAC_BIG if (gi == 0 and len(groups) > 1) else WS_INNER_FRAC,
                              seed=seed))
        if g0_first and gi == 0:
            done[0] = min(chunk, left)
            runs[0]["steps"](done[0])
    from ..utils.timing import hmark
    hmark("ws_groups_ready")
    # HFENS_WS_EVENTS=1 (diagnostic): device events per group after every enqueued chunk, read by
    # scripts/probes/ws_events.py (event time − the batch's start event, no profiler attached)
    evs = None
    if WS_EVENTS and cuda:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record(caller)
        evs = dict(start=ev0, rounds=[[] for _ in runs])

        def _mark(gi, r):
            e = torch.cuda.Event(enable_timing=True)
            e.record(r["side"] if r["side"] is not None else caller)
            evs["rounds"][gi].append(e)
    if sync:
        if after_first is not None:
            after_first()
        runs[0]["sync_rounds"](steps_per_check)
    else:
        # no host synchronisation: WS_ROUNDS_AHEAD rounds are enqueued at once (finished problems
        # return from each launch at once), so the caller's other streams are launched meanwhile;
        # a batch still unconverged after them reports err and is re-solved synchronously by
        # finish_svc_batch.  The groups' rounds are enqueued interleaved in chunks, so every
        # group's stream starts within one chunk of host launch time.
        while any(d < left for d in done):
            for gi, r in enumerate(runs):
                k = min(chunk, left - done[gi])
                if k > 0:
                    r["steps"](k)
                    done[gi] += k
                    if evs is not None:
                        _mark(gi, r)
            if after_first is not None:
                after_first()
                after_first = None
            hmark("ws_chunk")
        if after_first is not None:
            after_first()
    for gi, r in enumerate(runs):
        r["finish"]()
        if evs is not None:
            _mark(gi, r)
        # the run's closures refer back to its dict (finish sets out["err"]): drop them, so the runs
        # kept by the lazy statistics below are freed by reference counting, not by a full GC
        r["finish"] = r["steps"] = r["sync_rounds"] = None
    if evs is not None:
        LAST_WS_EVENTS.clear()
        LAST_WS_EVENTS.update(evs, chunk=chunk if not sync else None)
    # split join (deps_out given, no graphs): the caller's stream does NOT wait for every group —
    # the consumers wait for the groups of the problems they read (deps_out["wait"]); everything
    # that needs the whole batch (ρ / iterations of every problem, the error word) is assembled on
    # the first group's stream after it has waited for the others (deps_out["join"]).  The stacking
    # fit's Platt / out-of-fold / meta chain reads only the Platt-CV and fold problems, so it no
    # longer waits for the refit's final problem — the longest one (profiles/r6_headline.md).
    split = deps_out is not None and not use_graph and len(runs) > 1 and cuda
    for r in runs:
        if r["side"] is not None:
            if not split:
                caller.wait_stream(r["side"])
            for t in (alpha, G, zn, keys, zcat, r["rho"], r["iters"], r["idx_dev"]) + ((seed,) if seed is not None else ()):
                t.record_stream(r["side"])
    if use_graph:
        # the solution leaves the workspace: the next fit's rounds may overwrite it while this
        # fit's models are still being extracted on another stream
        alpha = alpha.clone()
    if len(runs) == 1:
        rho, iters, err = runs[0]["rho"], runs[0]["iters"], runs[0]["err"]
    elif split:
        ev_of = []
        for r in runs:
            ev = torch.cuda.Event()
            ev.record(r["side"] if r["side"] is not None else caller)
            ev_of.append(ev)
        J = runs[0]["side"] if runs[0]["side"] is not None else caller
        for gi, ev in enumerate(ev_of):
            if runs[gi]["side"] is not J:
                J.wait_event(ev)
        with torch.cuda.stream(J):
            rho = torch.empty(P, dtype=torch.float64, device=device)
            iters = torch.empty(P, dtype=torch.int32, device=device)
            for r in runs:
                rho.index_copy_(0, r["idx_dev"], r["rho"])
                iters.index_copy_(0, r["idx_dev"], r["iters"])
            err = torch.stack([r["err"] for r in runs]).amax().reshape(1)
            join_ev = torch.cuda.Event()
            join_ev.record(J)
        for t in (rho, iters, err):
            t.record_stream(caller)
        run_of = np.empty(P, dtype=np.int64)
        for gi, r in enumerate(runs):
            run_of[r["idx"]] = gi

        def wait(stream, problems):
            """Make ``stream`` wait for the groups holding ``problems`` (indices into live)."""
            for gi in sorted({int(run_of[k]) for k in problems}):
                stream.wait_event(ev_of[gi])

        def rho_for(stream, problems):
            """ρ of every problem [P] on ``stream``, valid for the groups holding ``problems``."""
            gis = sorted({int(run_of[k]) for k in problems})
            with torch.cuda.stream(stream):
                rr = torch.zeros(P, dtype=torch.float64, device=device)
                for gi in gis:
                    stream.wait_event(ev_of[gi])
                    runs[gi]["rho"].record_stream(stream)
                    rr.index_copy_(0, runs[gi]["idx_dev"], runs[gi]["rho"])
            return rr
        deps_out.update(wait=wait, rho_for=rho_for, join=J, join_ev=join_ev)
    else:
        rho = torch.empty(P, dtype=torch.float64, device=device)
        iters = torch.empty(P, dtype=torch.int32, device=device)
        for r in runs:
            rho.index_copy_(0, r["idx_dev"], r["rho"])
            iters.index_copy_(0, r["idx_dev"], r["iters"])
        err = None if sync else torch.stack([r["err"] for r in runs]).amax().reshape(1)

    def stats():   # read back only when someone looks (tests, bench diagnostics)
        if cuda:
            torch.cuda.synchronize(device)   # (the groups' streams need not be joined to the caller's)
        order = np.concatenate([r["idx"] for r in runs])
        inv = np.empty_like(order)
        inv[order] = np.arange(order.shape[0])
        parts = [r["stats"]() for r in runs]
        out = {k: np.concatenate([p[k] for p in parts])[inv]
               for k in ("outer", "inner", "gap", "cyc_select", "cyc_build", "cyc_inner", "cyc_p0", "cyc_p1", "cyc_p2")}
        ph = [p["phases"] for p in parts]
        out.update(q=Q, groups=[list(map(int, r["idx"])) for r in runs],
                   phases=np.concatenate(ph)[inv] if all(x is not None for x in ph) else None)
        return out
    LAST_WS_STATS.set_thunk(stats)
    LAST_SMO_INFO.clear()
    LAST_SMO_INFO.update(problems=P, max_l=int(ml), solver="ws", q=Q, ws_groups=len(runs),
                         ws_kc=kc_all)
    return alpha, rho, iters, err


def _ws_group(E, live, idx, zcat, zoffs, aoffs, F, device, eps, max_outer, max_inner, s, side,
              zn, alpha, G, keys, hist, n, Q, Fp2, kc=False, gi=None, cap_stream=None, frac=None, seed=None):
    """State of the problems ``live[idx]``, whose rounds go on stream ``s`` (per-problem state is
    group-local; the per-point arrays are the shared ones, addressed by each problem's absolute
    offset).  Returns closures: ``steps(k)`` enqueues k rounds, ``sync_rounds(chunk)`` runs
    host-checked rounds until every problem is done, ``finish()`` enqueues the ρ / statistics pass."""
    P = len(idx)
    frac = WS_INNER_FRAC if frac is None else frac
    arr = np.zeros(P, _WS_DT)
    # (column-wise: a per-record tuple assignment costs ~1.5 µs each, ≈ 0.3 ms for the cascade's
    # ~200 parts on the host critical path)
    ii = np.asarray(idx, dtype=np.int64)
    arr["zoff"] = np.asarray(zoffs, dtype=np.int64)[ii]
    arr["aoff"] = np.asarray(aoffs, dtype=np.int64)[ii]
    if isinstance(live, _PartSet):
        arr["l"], arr["npos"] = live.l[ii], live.npos[ii]
        arr["Cp"], arr["Cn"] = live.Cp[ii], live.Cn[ii]
        arr["ngl2e"] = -live.gamma[ii] * 1.4426950408889634
        fits = live.fit[ii]
    else:
        ps = [live[j] for j in idx]
        arr["l"] = [p.l for p in ps]
        arr["npos"] = [p.npos for p in ps]
        arr["Cp"] = [p.Cp for p in ps]
        arr["Cn"] = [p.Cn for p in ps]
        arr["ngl2e"] = [-p.gamma * 1.4426950408889634 for p in ps]
        fits = [p.fit for p in ps]
    max_l = int(arr["l"].max())
    ctx = (lambda: torch.cuda.stream(side)) if side is not None else contextlib.nullcontext
    out = dict(side=side, idx=np.asarray(idx, dtype=np.int64), err=None)
    graph = gi is not None
    with ctx():
        if graph:
            from .. import runtime

            def buf(name, numel, dtype):
                t = runtime.workspace(device, f"ws_g{gi}_{name}", numel, dtype)
                t.zero_()
                return t
            host = torch.from_numpy(arr.view(np.uint8).copy()).pin_memory()
            pdev = runtime.workspace(device, f"ws_g{gi}_pdev", host.numel(), torch.uint8)
            pdev.copy_(host, non_blocking=True)
        else:
            def buf(name, numel, dtype):
                return torch.zeros(numel, dtype=dtype, device=device)
            pdev = _dev_struct(arr, device)
            host = None
        if _GAMMA_CTX[0] is not None:
            _GAMMA_CTX[0].patch(pdev, _WS_DT, "ngl2e", fits)
        states = buf("states", P * _WS_STATE_BYTES // 4, torch.int32)
        wsz = buf("wsz", P * Fp2 * Q, torch.float32)
        wsn = buf("wsn", P * Q, torch.float32)
        wdc = buf("wdc", P * Q, torch.float32)
        wsprev = buf("wsprev", P * (Q // 2), torch.int32)
        wsidx = buf("wsidx", P * Q, torch.int32)
        wprof = torch.zeros(P * 6, dtype=torch.int64, device=device) if PROFILE_WS else None
        gkey = buf("gkey", 2 * P, torch.int64)
        cand = None
        if kc:
            nc_out = np.zeros(1, dtype=np.int64)
            E.ws_kc_cand_len(max_l, nc_out.ctypes.data)
            if int(nc_out[0]) > 0:   # large problems: per-block candidate lists (svm_ws.hip ws_cand_kernel)
                cand = buf("cand", 3 * P * int(nc_out[0]), torch.int32)
        rho = torch.empty(P, dtype=torch.float64, device=device)
        iters = torch.empty(P, dtype=torch.int32, device=device)
        inner = torch.empty(P, dtype=torch.int64, device=device)
        gap = torch.empty(P, dtype=torch.float64, device=device)
        E.ws_init(pdev.data_ptr(), P, max_l, zcat.data_ptr(), F, zn.data_ptr(), alpha.data_ptr(), G.data_ptr(),
                  states.data_ptr(), keys.data_ptr(), n, hist.data_ptr(), gkey.data_ptr(), s)
        if seed is not None:
            E.ws_seed(pdev.data_ptr(), P, max_l, zcat.data_ptr(), F, zn.data_ptr(), seed.data_ptr(),
                      alpha.data_ptr(), G.data_ptr(), keys.data_ptr(), n, gkey.data_ptr(), s)
            out["seed"] = seed
        out["idx_dev"] = _to_dev(out["idx"], device)
    done_view = states.view(P, _WS_STATE_BYTES // 4)[:, 0]

    def steps(k):
        if graph:
            # one captured graph per (group, shape, buffers, round count); replayed on the group's stream
            key = (gi, P, max_l, F, n, k, eps, max_outer, max_inner, frac,
                   tuple(int(t.data_ptr()) for t in (pdev, zcat, zn, alpha, G, states, wsz, wsn, wdc, wsprev,
                                                        keys, gkey)), int(cand.data_ptr()) if cand is not None else 0)
            g = _WS_GRAPHS.get(key)
            if g is None:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(cap_stream):
                    g.capture_begin(capture_error_mode="thread_local")
                    try:
                        launch(k)
                    finally:
                        g.capture_end()
                _WS_GRAPHS[key] = g
                while len(_WS_GRAPHS) > 24:
                    _WS_GRAPHS.pop(next(iter(_WS_GRAPHS)))
            with torch.cuda.stream(cap_stream):
                g.replay()
            return
        launch(k)

    def launch(k):
        if kc:
            E.ws_steps_kc(pdev.data_ptr(), P, max_l, zcat.data_ptr(), F, zn.data_ptr(), alpha.data_ptr(),
                          G.data_ptr(), states.data_ptr(), wsz.data_ptr(), wsn.data_ptr(), wdc.data_ptr(),
                          wsprev.data_ptr(), keys.data_ptr(), n, gkey.data_ptr(),
                          cand.data_ptr() if cand is not None else 0, eps, max_outer, max_inner,
                          frac, k, wprof.data_ptr() if wprof is not None else 0, s)
            return
        E.ws_steps(pdev.data_ptr(), P, max_l, zcat.data_ptr(), F, zn.data_ptr(), alpha.data_ptr(), G.data_ptr(),
                   states.data_ptr(), wsz.data_ptr(), wsn.data_ptr(), wdc.data_ptr(), wsprev.data_ptr(),
                   wsidx.data_ptr(), keys.data_ptr(), n, gkey.data_ptr(), eps, max_outer, max_inner, frac,
                   k, wprof.data_ptr() if wprof is not None else 0, WS_THREADS, Q, s)

    def sync_rounds(steps_per_check):
        outer = 0
        chunk = steps_per_check or 24   # one host check after the first 24 rounds, then every 8
        while outer < max_outer:
            steps(chunk)
            outer += chunk
            chunk = steps_per_check or 8
            if bool((done_view != 0).all()):
                break

    def finish():
        with ctx():
            if not _WS_SYNC[0]:
                out["err"] = (done_view == 0).any().to(torch.int32).reshape(1)
            E.ws_finalize(pdev.data_ptr(), P, states.data_ptr(), alpha.data_ptr(), G.data_ptr(), rho.data_ptr(),
                          iters.data_ptr(), inner.data_ptr(), gap.data_ptr(), s)

    def stats():
        cyc = states.view(P, _WS_STATE_BYTES // 4)[:, 10:22].cpu().contiguous().view(torch.int64).numpy()
        return dict(outer=iters.cpu().numpy(), inner=inner.cpu().numpy(), gap=gap.cpu().numpy(),
                    cyc_select=cyc[:, 0], cyc_build=cyc[:, 1], cyc_inner=cyc[:, 2],
                    cyc_p0=cyc[:, 3], cyc_p1=cyc[:, 4], cyc_p2=cyc[:, 5],
                    phases=wprof.view(P, 6).cpu().numpy() if wprof is not None else None)
    out.update(rho=rho, iters=iters, steps=steps, sync_rounds=sync_rounds, finish=finish, stats=stats,
               keep=(pdev, states, wsz, wsn, wdc, wsprev, wsidx, gkey, wprof, inner, gap, cand, host))
    return out


class _LazyStats(dict):
    """A dict filled on first read from a thunk (device statistics read back only if used)."""

    def set_thunk(self, f):
        self.clear()
        self._f = f

    def _fill(self):
        f = getattr(self, "_f", None)
        if f is not None:
            self._f = None
            super().update(f())

    def __getitem__(self, k):
        self._fill()
        return super().__getitem__(k)

    def get(self, k, d=None):
        self._fill()
        return super().get(k, d)

    def __contains__(self, k):
        self._fill()
        return super().__contains__(k)


LAST_WS_STATS = _LazyStats()
LAST_SMO_PROF: dict = {}
LAST_SMO_INFO: dict = {}
PROFILE_SMO = os.environ.get("HFENS_PROFILE_SMO", "0") == "1"
PROFILE_COOP = os.environ.get("HFENS_PROFILE_COOP", "0") == "1"   # in-kernel phase counters of the cooperative SMO
PROFILE_WS = os.environ.get("HFENS_PROFILE_WS", "0") == "1"       # phase counters (q=1024: svm_ws.hip built with -DHFENS_WS_STAMPS; K-cached: a stamped instance)


def assign_problems(sizes, world: int) -> List[int]:
    """Owner rank of every SMO problem, identical on every rank.  On a GPU the problems of one rank
    run side by side (one CU each), so a rank's time is its LARGEST problem's (the sequential pair
    loop), not the sum: the largest problem — the fit's critical path — gets rank 0 to itself
    (nothing else competes for its rank's CUs, HBM or host launches), and the others are spread
    longest-first onto the least-loaded of ranks 1 … W−1 (cost ∝ points).  One rank: all on 0."""
    load = [0] * world
    owner = [0] * len(sizes)
    order = sorted(range(len(sizes)), key=lambda k: (-sizes[k], k))
    if world >= 2 and len(sizes) >= 2:
        owner[order[0]] = 0
        load[0] = sizes[order[0]]
        order, ranks = order[1:], range(1, world)
    else:
        ranks = range(world)
    for k in order:
        r = min(ranks, key=lambda r: (load[r], r))
        owner[k] = r
        load[r] += sizes[k]
    return owner


def _solve_distributed(solve_local, live, n_alpha, aoffs, device, group):
    """Task-parallel SMO (SURVEY.md §2.4 ensemble parallel, call site R9): rank r solves the
    problems ``assign_problems`` gives it; one SUM all-reduce of a zero-filled int64
    [α bits | ρ bits | iters | err count] vector gives every rank every solution.  Every α / ρ / iters
    entry has exactly one non-zero contributor and travels as its f64 BIT PATTERN (an f64
    sum would turn an owner's −0.0 into +0.0; an integer x + 0 = x for every pattern), so every rank
    holds the owner's bits; the last entry counts the ranks whose solve reported an error."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    owner = assign_problems([p.l for p in live], world)
    mine = [k for k in range(len(live)) if owner[k] == rank]
    P = len(live)
    flat = torch.zeros(n_alpha + 2 * P + 1, dtype=torch.int64, device=device)
    if mine:
        sub = [live[k] for k in mine]
        a_s, r_s, it_s, err_s = solve_local(sub)
        so = np.concatenate([[0], np.cumsum([p.l for p in sub])]).astype(np.int64)
        for i, k in enumerate(mine):
            flat[aoffs[k]:aoffs[k] + live[k].l] = a_s[so[i]:so[i + 1]].to(torch.float64).view(torch.int64)
        idx = _to_dev(np.asarray(mine, dtype=np.int64), device)
        flat[n_alpha:n_alpha + P].index_copy_(0, idx, r_s.to(torch.float64).reshape(-1).contiguous().view(torch.int64))
        flat[n_alpha + P:n_alpha + 2 * P].index_copy_(0, idx, it_s.to(torch.int64).reshape(-1))
        if err_s is not None:
            flat[n_alpha + 2 * P:] += (err_s.to(torch.float64).reshape(-1) != 0).any().to(torch.int64)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    bits = flat[:n_alpha + P].view(torch.float64)
    return (bits[:n_alpha], bits[n_alpha:], flat[n_alpha + P:n_alpha + 2 * P].to(torch.int32),
            flat[n_alpha + 2 * P:].to(torch.float64))


# Cascade seed (the critical problem's pair count).  Every working-set problem of
# ≥ CASCADE_MIN points is split into disjoint class-stratified parts of ≈ CASCADE_PART points, each
# solved as an SVC with the SAME per-class C to the loose tolerance CASCADE_EPS (q = 512: half the
# slots per pair); the concatenated part solutions satisfy the full problem's box and equality
# constraints, so they are a feasible warm start, and the full problem is then solved from there to
# libsvm's eps by the same rule — same dual, same KKT stopping test, a different pair path (α agrees
# to O(eps), as with any working-set solve).  Host simulation of the bench's 10k refit problem
# (scripts/probes/ws_cascade_sim.py, 8 parts, part eps 0.1): 778 part pairs + 4,954 seeded pairs
# (22 rounds) vs 8,442 cold (37 rounds); decision values differ by 1.7e-3 from the cold solve, the
# same as cold q = 512 vs q = 1024 (1.5e-3).
CASCADE = os.environ.get("HFENS_SVM_CASCADE", "1") != "0"
CASCADE_MIN = int(os.environ.get("HFENS_SVM_CASCADE_MIN", "4096"))
CASCADE_PART = int(os.environ.get("HFENS_SVM_CASCADE_PART", "1600"))
# part tolerance 0.3 (round 6 sweep on one box each, profiles/r6_runs/r6v, r6w: 17.28 / 17.18 ms / fit vs
# 17.9 / 18.0 / 18.1 at 0.1; the looser parts end sooner and the seeded solve needs fewer pairs,
# 4,892 vs 5,131 on the critical problem)
CASCADE_EPS = float(os.environ.get("HFENS_SVM_CASCADE_EPS", "0.3"))
CASCADE_Q = int(os.environ.get("HFENS_SVM_CASCADE_Q", "512"))
# also seed the K-cached solver (problems past 16k points: candidate-list rounds of q = 256)
CASCADE_KC = os.environ.get("HFENS_SVM_CASCADE_KC", "1") != "0"
# working-set rounds the parts get (a fixed budget: every round is enqueued ahead without a host
# check, so rounds past the parts' convergence are launches the full solve waits on; a part stopped
# by the budget is still feasible and still seeds)
CASCADE_ROUNDS = int(os.environ.get("HFENS_SVM_CASCADE_ROUNDS", "8"))
LAST_CASCADE: dict = {}


def cascade_split(l: int, npos: int) -> int:
    """Number of cascade parts of a problem of l points (npos positive); 0 = solved cold."""
    if l < CASCADE_MIN or CASCADE_PART <= 0:
        return 0
    P = max(2, int(round(l / CASCADE_PART)))
    return P if (npos >= P and l - npos >= P) else 0


def cascade_parts(p: _Prob) -> List[np.ndarray]:
    """Positions (in problem order: positives first) of p's parts, or [] when p is solved cold:
    part j holds every P-th positive and every P-th negative from j on (the host mirror of
    stackdev.hip cascade_where_kernel)."""
    P = cascade_split(p.l, p.npos)
    nneg = p.l - p.npos
    return [np.concatenate([np.arange(j, p.npos, P), p.npos + np.arange(j, nneg, P)]) for j in range(P)]


class _Part:
    """A cascade part's solver record (its rows are gathered on the device, never listed on the host)."""
    __slots__ = ("fit", "fold", "l", "npos", "Cp", "Cn", "gamma")

    def __init__(self, fit, fold, l, npos, Cp, Cn, gamma):
        self.fit, self.fold, self.l, self.npos, self.Cp, self.Cn, self.gamma = fit, fold, l, npos, Cp, Cn, gamma


class _PartSet:
    """The cascade's parts as arrays (one entry per part): built with a few numpy operations instead
    of ≈ 200 Python records per fit on the host path to the parts' launch.  Indexing yields a
    :class:`_Part`; :func:`_ws_group` and :func:`_solve_ws` read the arrays directly."""

    def __init__(self, fit, fold, l, npos, Cp, Cn, gamma):
        self.fit, self.fold, self.l, self.npos, self.Cp, self.Cn, self.gamma = fit, fold, l, npos, Cp, Cn, gamma
        self.max_l = int(l.max()) if l.shape[0] else 0

    def __len__(self):
        return int(self.l.shape[0])

    def __getitem__(self, k):
        return _Part(int(self.fit[k]), int(self.fold[k]), int(self.l[k]), int(self.npos[k]), float(self.Cp[k]),
                     float(self.Cn[k]), float(self.gamma[k]))

    def __iter__(self):
        return (self[k] for k in range(len(self)))


def _max_l(live) -> int:
    return live.max_l if isinstance(live, _PartSet) else max(p.l for p in live)


def _cascade_tables(live, aoffs):
    """(parts table [n_parts, 7] int64: start, length, parent offset, P, j, parent npos, part npos;
    the parts as a :class:`_PartSet`), or None when no problem is split.  :func:`cascade_split`,
    vectorised: P = max(2, round(l / CASCADE_PART)) parts (round half to even, as Python's round)
    when l ≥ CASCADE_MIN and both classes have ≥ P points, else 0 (solved cold)."""
    K = len(live)
    l = np.fromiter((p.l for p in live), np.int64, K)
    npos = np.fromiter((p.npos for p in live), np.int64, K)
    if CASCADE_PART > 0:
        P = np.maximum(2, np.rint(l / CASCADE_PART).astype(np.int64))
        P = np.where((l >= CASCADE_MIN) & (npos >= P) & (l - npos >= P), P, 0)
    else:
        P = np.zeros(K, np.int64)
    if not P.any():
        return None
    # part j of problem k takes ⌈(npos − j) / P⌉ positives and ⌈(nneg − j) / P⌉ negatives
    kk = np.repeat(np.arange(K), P)
    j = np.arange(kk.shape[0]) - np.repeat(np.cumsum(P) - P, P)
    Pk, nk = P[kk], npos[kk]
    cp = (nk - j + Pk - 1) // Pk
    cn = (l[kk] - nk - j + Pk - 1) // Pk
    ln = cp + cn
    start = np.cumsum(ln) - ln
    tab_np = np.stack([start, ln, np.asarray(aoffs[:K], dtype=np.int64)[kk], Pk, j, nk, cp], axis=1)
    f64 = np.float64
    parts = _PartSet(np.fromiter((p.fit for p in live), np.int64, K)[kk],
                     np.fromiter((p.fold for p in live), np.int64, K)[kk], ln, cp,
                     np.fromiter((p.Cp for p in live), f64, K)[kk], np.fromiter((p.Cn for p in live), f64, K)[kk],
                     np.fromiter((p.gamma for p in live), f64, K)[kk])
    return tab_np, parts


def _cascade_seed(E, live, zcat, aoffs, F, device, s, max_iter_cap=None):
    """The feasible warm start of every problem (zeros for problems solved cold), or None.  The
    parts' point lists are built on the device (cascade_where) and their features gathered from the
    parents' rows in ``zcat`` — the host only counts."""
    ct = _cascade_tables(live, aoffs)
    if ct is None:
        return None
    tab_np, parts = ct
    where = torch.empty(int(tab_np[:, 1].sum()), dtype=torch.int64, device=device)
    E.cascade_where(_to_dev(tab_np.reshape(-1), device).data_ptr(), len(parts), int(tab_np[:, 1].max()),
                    where.data_ptr(), s)
    zpart = zcat.index_select(0, where)
    po = np.concatenate([[0], np.cumsum(tab_np[:, 1])]).tolist()
    a_parts, _, _, _ = _solve_ws(E, parts, zpart, po[:-1], po, F, device, CASCADE_EPS, CASCADE_ROUNDS, s,
                                 q=CASCADE_Q if ws_q(F) == 1024 else None, groups=1)
    from ..utils.timing import dmark
    dmark("svc_parts_done")
    LAST_CASCADE.clear()
    LAST_CASCADE.update(parts=len(parts), stats=LAST_WS_STATS._f)   # read lazily (device stats)
    seed = torch.zeros(aoffs[-1], dtype=torch.float64, device=device)
    # (a part solve stopped by its round budget is still feasible: it seeds)
    seed.index_copy_(0, where, a_parts)
    return seed


def _solve_device(probs: List[_Prob], Zs, device, eps, max_iter_cap=None, group=None, oof_items=None,
                  platt_prep=None):
    from .. import ops
    E = ops.ext()
    s = ops.stream_ptr(device)
    live = [p for p in probs if p.rows is not None]
    F = Zs[0].shape[1]
    LAST_SMO_INFO.clear()
    zcat = _gather_rows(Zs, live, "rows", device)
    from ..utils.timing import hmark, dmark
    hmark("svc_gather")
    zoffs, aoffs = [], [0]
    for p in live:
        zoffs.append(aoffs[-1])
        aoffs.append(aoffs[-1] + p.l)
    aoffs_start = aoffs[:-1]
    max_l = max(p.l for p in live)
    solver = _pick_solver(max_l, F)
    solve = _solve_ws if solver == "ws" else _solve_exact
    # ---- label-only tables of the post-SMO launches, uploaded while the main rounds run — once
    # every group's first rounds are enqueued (TABLES_AFTER_FIRST; each in-stream upload queued
    # behind the whole SMO cost ≈ 30 µs on the critical path; ahead of the parts they delayed the
    # parts' enqueue, ahead of the main rounds the critical group's first round):
    # the signs of y·α, the Platt decision table (+ the stacking fit's out-of-fold rows,
    # ``oof_items``), the Platt kernel's maps
    platt = [(k, p) for k, p in enumerate(live) if p.fold >= 0]
    out = {}
    tabs = {}

    def prep_tables():
        sign_h = np.empty(aoffs[-1], dtype=np.float32)
        for k, p in enumerate(live):
            a0, l = aoffs_start[k], p.l
            sign_h[a0:a0 + p.npos] = 1.0
            sign_h[a0 + p.npos:a0 + l] = -1.0
        sign_d = _to_dev(sign_h, device)
        pre_dec = None
        if platt:
            oof = []
            # (``oof_items`` may be a callable: the caller's out-of-fold rows formed only now)
            oi = oof_items() if callable(oof_items) else oof_items
            if oi and not (SPLIT_JOIN and group is None):
                finals = {p.fit: k for k, p in enumerate(live) if p.fold < 0}
                oof = [(finals[f], Zt) for f, Zt in oi if f in finals]
                if len(oof) != len(oi):
                    oof = []
            hcat = _gather_rows(Zs, [p for _, p in platt], "held_rows", device)
            if oof:
                hcat = torch.cat([hcat] + [Zt.to(torch.float32) for _, Zt in oof]).contiguous()
            per = 1024
            S = (max_l + per - 1) // per
            dt = np.zeros(len(platt) + len(oof), _DEC_DT)
            hoff = 0
            for i, (k, p) in enumerate(platt):
                h = int(p.held_rows.shape[0])
                dt[i] = (zoffs[k], hoff, p.l, h, -p.gamma * 1.4426950408889634, per)
                hoff += h
            hoff_platt = hoff
            for i, (k, Zt) in enumerate(oof):
                h = int(Zt.shape[0])
                dt[len(platt) + i] = (zoffs[k], hoff, live[k].l, h, -live[k].gamma * 1.4426950408889634, per)
                hoff += h
            part = torch.zeros(hoff, S, dtype=torch.float32, device=device)
            ddev = _dev_struct(dt, device)
            if _GAMMA_CTX[0] is not None:
                _GAMMA_CTX[0].patch(ddev, _DEC_DT, "ngl2e", [p.fit for _, p in platt] + [live[k].fit for k, _ in oof])
            rowk = np.repeat(np.array([k for k, _ in platt], dtype=np.int32), dt["h"][:len(platt)].astype(np.int64))
            rowk_d = _to_dev(rowk, device)
            for i, (k, p) in enumerate(platt):
                out[("hoff", id(p))] = (int(dt[i]["hoff"]), int(dt[i]["h"]))
            if platt_prep is not None:
                out["platt_prep"] = platt_prep({id(p): out[("hoff", id(p))] for _, p in platt})
            pre_dec = dict(oof=oof, oi=oi, hcat=hcat, S=S, dt=dt, hoff=hoff, hoff_platt=hoff_platt, part=part, ddev=ddev,
                           rowk=rowk_d)
        tabs.update(sign_d=sign_d, pre_dec=pre_dec)
        hmark("svc_tables")
    deps: dict = {}
    if group is None:
        kw = {}
        if solver == "ws" and CASCADE and (CASCADE_KC or not ws_kc(F, max_l)):
            seed = _cascade_seed(E, live, zcat, aoffs, F, device, s, max_iter_cap)
            if seed is not None:
                kw["seed"] = seed
                hmark("svc_cascade_seeded")
        if solver == "ws" and SPLIT_JOIN:
            kw["deps_out"] = deps
        if solver == "ws" and TABLES_AFTER_FIRST:
            # (built while the device runs the first rounds, off the critical group's enqueue)
            kw["after_first"] = prep_tables
        else:
            prep_tables()
        alpha, rho, iters, err = solve(E, live, zcat, zoffs, aoffs, F, device, eps, max_iter_cap, s, **kw)
    else:
        def solve_local(sub):
            zsub = _gather_rows(Zs, sub, "rows", device)
            so = [0]
            for p in sub:
                so.append(so[-1] + p.l)
            kw = {}
            if solver == "ws" and CASCADE and (CASCADE_KC or not ws_kc(F, max(p.l for p in sub))):
                seed = _cascade_seed(E, sub, zsub, so, F, device, s, max_iter_cap)
                if seed is not None:
                    kw["seed"] = seed
            return solve(E, sub, zsub, so[:-1], so, F, device, eps, max_iter_cap, s, **kw)
        prep_tables()
        alpha, rho, iters, err = _solve_distributed(solve_local, live, aoffs[-1], aoffs, device, group)
    out["smo_err"] = err
    J = deps.get("join")
    if J is not None:
        out["_deps"] = deps     # (consumers wait for the groups they read; finish joins them all)
    for k, p in enumerate(live):
        a0 = aoffs_start[k]
        out[id(p)] = (alpha[a0:a0 + p.l], rho[k], iters[k])
    # early read-back of what the final models' bookkeeping needs from the SMO alone (support masks,
    # ρ, iterations, the error word), queued right behind the SMO: finish_svc_batch extracts the
    # support vectors while the Platt and out-of-fold kernels still run, then reads only (A, B)
    fin = sorted((p.fit, k) for k, p in enumerate(live) if p.fold < 0)
    if EARLY_READ and fin and len({f for f, _ in fin}) == len(fin):
        f64 = torch.float64
        ks = [k for _, k in fin]
        # (split join: on the joining stream, behind every group)
        with (torch.cuda.stream(J) if J is not None else contextlib.nullcontext()):
            kidx = _to_dev(np.array(ks, dtype=np.int64), device)
            parts = ([(alpha[aoffs_start[k]:aoffs_start[k] + live[k].l] > 0).to(f64) for k in ks]
                     + [rho.index_select(0, kidx).to(f64).reshape(-1), iters.index_select(0, kidx).to(f64).reshape(-1)]
                     + ([err.to(f64).reshape(-1).abs().max().reshape(1)] if err is not None else []))
            early_dev = torch.cat(parts)
            early_host, ev = stage(early_dev)     # (finite once landed: polled by finish_svc_batch)
        out["_early"] = dict(host=early_host, ev=ev, ids=[id(live[k]) for k in ks], has_err=err is not None,
                             keep=early_dev)
    # y·α of every problem in f32 (the decision kernels' coefficients), kept with the problems' rows
    # for the held-out decisions below and the stacking trainer's device OOF (enqueue_svc_oof)
    # (the signs built on the host and uploaded in one copy, before the rounds)
    sign_d, pre_dec = tabs["sign_d"], tabs["pre_dec"]
    rho_pl = rho
    if J is not None:
        # the Platt decisions read only the Platt-CV problems: wait for their groups alone
        cur = torch.cuda.current_stream(device)
        deps["wait"](cur, [k for k, _ in platt])
        rho_pl = deps["rho_for"](cur, [k for k, _ in platt])
    coef = (sign_d * alpha.to(torch.float32)).contiguous()
    out["_dec"] = dict(zcat=zcat, coef=coef, F=F, zoff={id(p): zoffs[k] for k, p in enumerate(live)},
                       sign=sign_d, alpha=alpha, kof={id(p): k for k, p in enumerate(live)})
    # ---- Platt held-out decision values of every CV sub-model: one batched launch — with the
    # stacking fit's out-of-fold rows (``oof_items``: [(fit f, fold-f-scaled rows)], decided by fit f's
    # final problem) in the SAME launch, so enqueue_svc_oof needs no decision launch of its own
    if pre_dec is not None:
        pdd = pre_dec
        dmark("svc_smo_done")
        zsv, csv, cnt = _sv_compact(E, zcat, coef, F, pdd["ddev"], len(pdd["dt"]), device, s)
        E.svm_dec_batch(zsv.data_ptr(), csv.data_ptr(), pdd["hcat"].data_ptr(), F, pdd["ddev"].data_ptr(),
                        len(pdd["dt"]), int(pdd["dt"]["h"].max()), pdd["S"], pdd["part"].data_ptr(),
                        cnt.data_ptr() if cnt is not None else 0, s)
        if pdd["oof"]:
            out["oof_pre"] = dict(ids=[(f, id(Zt)) for f, Zt in pdd["oi"]], part=pdd["part"], hoff0=pdd["hoff_platt"],
                                  hoff=pdd["hoff"] - pdd["hoff_platt"])
        dmark("svc_platt_dec")
        # the decision values are assembled inside the Platt kernel from these partials (row r of
        # part: problem rowk[r]'s held-out point, d = −(Σ part[r] − ρ))
        out["platt_src"] = dict(part=pdd["part"], S=pdd["S"], rowk=pdd["rowk"],
                                rho=rho_pl.to(torch.float64).contiguous(), keep=(pdd["hcat"], pdd["ddev"], zsv, csv, cnt))
    return out


def _solve_host(probs: List[_Prob], Zs, eps, max_iter_cap=None, group=None):
    live = [p for p in probs if p.rows is not None]

    def solve_local(sub):
        alphas, rhos, its = [], [], []
        for p in sub:
            Zp = Zs[p.fit][torch.as_tensor(p.rows)].double().cpu().numpy()
            K = _gram_host(Zp, p.gamma)
            l = K.shape[0]
            mi = max(10_000_000, 100 * l) if max_iter_cap is None else max_iter_cap
            a, r, it = _smo_host(K, p.npos, p.Cp, p.Cn, eps, mi)
            alphas.append(torch.as_tensor(a))
            rhos.append(r)
            its.append(it)
        return (torch.cat(alphas) if alphas else torch.zeros(0, dtype=torch.float64),
                torch.tensor(rhos, dtype=torch.float64), torch.tensor(its, dtype=torch.int64), None)

    aoffs = [0]
    for p in live:
        aoffs.append(aoffs[-1] + p.l)
    if group is None:
        alpha, rho, iters, _ = solve_local(live)
    else:
        alpha, rho, iters, _ = _solve_distributed(solve_local, live, aoffs[-1], aoffs, torch.device("cpu"), group)
    out = {}
    for k, p in enumerate(live):
        out[id(p)] = (alpha[aoffs[k]:aoffs[k + 1]].clone(), rho[k].clone(), iters[k].clone())
    return out


# ----------------------------------------------------------------------------- public
def fit_svc_batch(svcs, Zs: List[torch.Tensor], ys: List[torch.Tensor], max_iter_cap=None, group=None):
    """Fit ``svcs[f]`` on (already scaled) ``Zs[f]`` with labels ``ys[f]`` ∈ {0,1}."""
    return finish_svc_batch(launch_svc_batch(svcs, Zs, ys, max_iter_cap, group=group))


# Exact vs large-problem path (``svc_lowrank``: Nyström reduced-set SVC, interior-point dual).
# GPU: the working-set SMO needs O(n) memory (no Gram), and its candidate-list selection handles any
# size, so "auto" keeps every problem exact up to EXACT_MAX_POINTS — the measured crossover
# (scripts/probes/svc_crossover.py, profiles/r4_svc_crossover.md: one probability fit, exact vs
# Nyström 0.17 vs 1.56 s at 40k rows, 0.81 vs 1.55 s at 100k, 3.05 vs 1.94 s at 200k, 6.98 vs
# 2.04 s at 300k: exact time grows as l^1.9, so the two cross near 150k); features past the K-cached kernel's
# range (F > 24) keep the one-workgroup selector's 32,768-point limit.  Host (CPU): the exact solver
# stores every problem's Gram, so it stays below EXACT_HOST_MAX points and GRAM_BUDGET bytes.
EXACT_MAX_POINTS = int(os.environ.get("HFENS_SVM_EXACT_MAX", "150000"))
# the final solves' support masks / ρ / iterations read back right behind the SMO (before the Platt
# kernels), so finish_svc_batch's support extraction overlaps them (same-box A/B of the headline:
# within its ±0.7 ms run-to-run spread, scripts/probes/gpu_r4an.sh, profiles/r4_runs/early_read_ab.log)
EARLY_READ = os.environ.get("HFENS_SVC_EARLY_READ", "1") != "0"
# split join of the working-set groups (_solve_ws deps_out): the Platt decisions and the stacking
# fit's out-of-fold column wait only for the groups of the problems they read, not for the refit's
# final problem (the longest, whose model is only needed at the end)
# (measured, profiles/r6_runs/r6r: no gain on the headline — the Platt-CV groups end within
# ≈ 0.1 ms of the refit's 10k problem — so it is off by default: 18.07 / 17.79 vs 17.92 / 18.11 ms)
SPLIT_JOIN = os.environ.get("HFENS_SVM_SPLIT_JOIN", "0") == "1"
# the post-SMO label-only tables built once every working-set group's first rounds are enqueued
# ("0": before the main rounds, behind the cascade parts)
TABLES_AFTER_FIRST = os.environ.get("HFENS_SVC_TABLES_AFTER_FIRST", "1") == "1"
EXACT_HOST_MAX = int(os.environ.get("HFENS_SVM_EXACT_HOST_MAX", "32768"))
GRAM_BUDGET = float(os.environ.get("HFENS_SVM_GRAM_BUDGET", str(96 << 30)))


def use_lowrank(sizes, F: int = 17, device_type: str = "cpu") -> bool:
    if SOLVER == "lowrank":
        return True
    if SOLVER in ("exact", "ws"):
        return False
    m = max(sizes)
    # problem sizes ≈ 0.8·l (Platt folds) and l (final) per fit
    gram = sum(4.0 * (5 * (0.8 * l) ** 2 + l * l) for l in sizes)
    if device_type == "cuda":
        # past the working-set kernel's feature budget the device solver is the stored-Gram one
        # (_pick_solver): its Grams must fit the budget too
        return (m > EXACT_MAX_POINTS or (F > WS_KC_MAX_F and m >= 32768)
                or (F > WS_MAX_F and gram > GRAM_BUDGET))
    return m > EXACT_HOST_MAX or gram > GRAM_BUDGET


class _GammaDev:
    """γ of every fit computed on the device (``svm_gamma``): the problem records built on the host
    carry a placeholder that :meth:`patch` overwrites on the device, so no host read of the scaled
    data's variance stands between the scaler and the SMO."""

    def __init__(self, Zs, device):
        from .. import ops
        K, F = len(Zs), int(Zs[0].shape[1])
        base = Zs[0]
        lens = [int(Z.shape[0]) for Z in Zs]
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        contiguous = all(Z.is_contiguous() and Z.dtype == torch.float64 for Z in Zs) and all(
            Zs[k].data_ptr() == base.data_ptr() + int(offs[k]) * F * 8 for k in range(K))
        Zc = base if contiguous else torch.cat([Z.to(torch.float64) for Z in Zs]).contiguous()
        self.offs = _to_dev(offs, device)
        self.gam = torch.empty(K, dtype=torch.float64, device=device)
        self.ngl = torch.empty(K, dtype=torch.float32, device=device)
        ops.ext().svm_gamma(Zc.data_ptr(), self.offs.data_ptr(), K, F, self.gam.data_ptr(), self.ngl.data_ptr(),
                            ops.stream_ptr(device))
        # read back right behind its kernel (pinned + event): resolve() waits for γ, not for the SMO
        self.host, self.ev = stage(self.gam)     # (polled by resolve: see landed)
        self.keep = [Zc]

    def patch(self, ddev: torch.Tensor, dtype: np.dtype, field: str, fits) -> None:
        from .. import ops
        fo = _to_dev(np.asarray(fits, dtype=np.int32), ddev.device)
        ops.ext().svm_patch_f32(ddev.data_ptr(), int(dtype.itemsize), int(dtype.fields[field][1]), len(fits),
                                fo.data_ptr(), self.ngl.data_ptr(), ops.stream_ptr(ddev.device))
        self.keep.append(fo)

    def resolve(self, all_probs, meta) -> None:
        """The host's γ (models, host mirrors): one small read, queued when γ was computed."""
        # (γ is finite unless the scaled rows are not: a non-finite γ waits out landed's budget,
        # then the event, then raises below)
        g = landed(self.host, self.ev).copy()
        if not np.isfinite(g).all():
            from ..utils.guards import NonFiniteError
            raise NonFiniteError("SVC.fit X: non-finite scaled value(s)")
        for p in all_probs:
            p.gamma = float(g[p.fit])
        for f, mt in enumerate(meta):
            mt["gamma"] = float(g[f])


_GAMMA_CTX: list = [None]


def launch_svc_batch(svcs, Zs: List[torch.Tensor], ys: List[torch.Tensor], max_iter_cap=None, group=None,
                     y_host=None, plan=None, gamma_dev: bool = False, oof_items=None) -> dict:
    """Everything up to the Platt sigmoid fits, enqueued on the current stream with no host
    synchronisation after the SMO launch (so the caller can overlap other work); complete
    with :func:`finish_svc_batch`.  ``group``: every rank holds the same (full) ``Zs``; the SMO
    problems are solved task-parallel over the ranks (:func:`assign_problems`) and their
    solutions all-reduced — one collective, issued from the calling thread.

    Fits above the exact solver's size/memory limits (:func:`use_lowrank`) are solved by the
    Nyström reduced-set SVC (:mod:`svc_lowrank`) instead, synchronously; with ``group`` fit ``f``
    is solved on rank ``f mod world`` and broadcast.

    ``y_host``: the fits' labels as host arrays (the caller already has them): the libsvm problem
    expansion then runs on the host while the device computes the guards and γ statistics, and
    only those are read back.

    ``gamma_dev`` (GPU, a ``plan`` of 0/1 labels, gamma='scale', the working-set solver): NO host
    read at all — γ is computed and patched into the problem records on the device
    (:class:`_GammaDev`), the labels' 0/1 guard ran in the plan, and the scaled rows' finite guard is
    the γ's own (read by :func:`finish_svc_batch`).  The stacking trainer uses it to enqueue the
    whole batch before the selected columns reach the host (pipeline.develop)."""
    from .. import ops
    if use_lowrank([int(y.numel()) for y in ys], int(Zs[0].shape[1]), Zs[0].device.type):
        from .svc_lowrank import fit_svc_lowrank_batch
        LAST_SMO_INFO.clear()
        LAST_SMO_INFO.update(solver="nystrom-ipm", problems=6 * len(svcs), max_l=max(int(y.numel()) for y in ys))
        if group is None:
            fit_svc_lowrank_batch(svcs, Zs, ys)
        else:
            from ..parallel.stack import broadcast_svc_fits
            import torch.distributed as dist
            world, rank = dist.get_world_size(group), dist.get_rank(group)
            mine = [f for f in range(len(svcs)) if f % world == rank]
            if mine:
                fit_svc_lowrank_batch([svcs[f] for f in mine], [Zs[f] for f in mine], [ys[f] for f in mine])
            broadcast_svc_fits(svcs, Zs, group)
        return dict(done=True, svcs=svcs)
    from ..utils import guards
    from ..utils.timing import hmark, dmark
    device = Zs[0].device
    cuda = Zs[0].is_cuda
    # ONE device→host read for everything the host bookkeeping needs: the finite / 0-1 guard
    # flags, the 'scale' gamma statistics and every fit's labels (the problem bookkeeping itself
    # is numpy on the host)
    sizes = [int(y.numel()) for y in ys]
    need_var = [svc.gamma == "scale" for svc in svcs]
    f64 = torch.float64
    pre = None
    if plan is not None and len(plan) == len(svcs) and all(int(p[0].shape[0]) == int(y.numel()) for p, y in zip(plan, ys)):
        pre = plan   # expanded ahead of time (plan_svc_problems), overlapped with earlier device work
        hmark("svc_expand_planned")
    gdev = None
    # (with ``group``, the task-parallel policy: every rank holds the same Zs, so every rank's γ
    # kernel computes the same bits)
    if (gamma_dev and cuda and pre is not None and all(need_var)
            and _pick_solver(max(int(p.l) for _, pr, _ in pre for p in pr), int(Zs[0].shape[1])) == "ws"):
        gdev = _GammaDev(Zs, device)
    parts = []
    if guards.ENABLED and gdev is None:
        parts.append(torch.stack([torch.isfinite(Z).all() for Z in Zs]).to(f64))
        parts.append(torch.stack([((y == 0) | (y == 1)).all() for y in ys]).to(f64))
    if any(need_var) and gdev is None:
        parts.append(torch.stack([Z.to(f64).var(unbiased=False) for Z in Zs]))
    if pre is not None:
        pass
    elif y_host is not None and all(((yh == 0.0) | (yh == 1.0)).all() for yh in y_host):
        # host labels: expand the problems now (γ filled in below), overlapping the device work
        pre = []
        for f, (svc, yh) in enumerate(zip(svcs, y_host)):
            y_np = np.asarray(yh, dtype=np.float64).reshape(-1)
            pre.append((y_np,) + _expand(f, y_np, None, _class_weights_host(svc, y_np), svc))
        hmark("svc_expand_early")
    else:
        parts.append(torch.cat([y.reshape(-1).to(f64) for y in ys]))
    host = torch.cat(parts).cpu().numpy() if parts else np.zeros(0)
    o = 0
    if guards.ENABLED and gdev is None:
        for f in range(len(Zs)):
            if host[f] == 0.0:
                guards.check_finite(Zs[f], f"SVC.fit X (fit {f})")
            if host[len(Zs) + f] == 0.0:
                guards.check_binary(ys[f], f"SVC.fit y (fit {f})")
        o = 2 * len(Zs)
    var = None
    if any(need_var) and gdev is None:
        var = host[o:o + len(Zs)]
        o += len(Zs)
    y_all = host[o:]
    hmark("svc_y_var_host")
    all_probs, meta = [], []
    off = 0
    for f, (svc, Z) in enumerate(zip(svcs, Zs)):
        if gdev is not None:
            gamma = 0.0          # (placeholder: the device records are patched, the host reads γ at finish)
        elif svc.gamma == "scale":
            v = float(var[f])
            gamma = 1.0 / (Z.shape[1] * v) if v != 0 else 1.0
        else:
            gamma = svc.resolve_gamma(Z)
        if pre is not None:
            _, pr, mt = pre[f]
            for p in pr:
                p.gamma = gamma
            mt["gamma"] = gamma
        else:
            y_np = y_all[off:off + sizes[f]]
            off += sizes[f]
            pr, mt = _expand(f, y_np, gamma, _class_weights_host(svc, y_np), svc)
        all_probs += pr
        meta.append(mt)
    hmark("svc_expand")
    eps = float(svcs[0].tol)
    args = (svcs, Zs, ys, max_iter_cap, group)
    pl = [f for f, svc in enumerate(svcs) if svc.probability]

    def platt_prep(hoff_of):
        """The Platt kernel's label-only tables (grouped-position → decision-partial row maps,
        per-fold constants, the fit records), uploaded before the SMO rounds."""
        arr = np.zeros(len(pl), _PLATT_DT)
        maps, consts, off = [], [0.0], 0
        for k, f in enumerate(pl):
            mt = meta[f]
            l = mt["l"]
            sm = np.full(l, -1, dtype=np.int32)
            for p in (q for q in all_probs if q.fit == f and q.fold >= 0):
                if p.rows is not None:
                    h0, h = hoff_of[id(p)]
                    sm[p.held] = np.arange(h0, h0 + h, dtype=np.int32)
                else:
                    consts.append(float(p.const))
                    sm[p.held] = -len(consts)
            arr[k] = (off, l, mt["n0"])
            maps.append(sm)
            off += l
        return dict(srcmap=_to_dev(np.concatenate(maps), device),
                    cdev=_to_dev(np.asarray(consts, dtype=np.float64), device), off=off,
                    pdev=_dev_struct(arr, device))
    _GAMMA_CTX[0] = gdev
    try:
        sol = (_solve_device(all_probs, Zs, device, eps, max_iter_cap, group, oof_items=oof_items,
                             platt_prep=platt_prep if pl else None) if cuda
               else _solve_host(all_probs, Zs, eps, max_iter_cap, group))
    finally:
        _GAMMA_CTX[0] = None
    hmark("svc_solve_enqueued")
    solver = LAST_SMO_INFO.get("solver")   # this batch's solver (the global is overwritten by later batches)
    # ---- Platt: held-out decision values per fit (grouped-position order), then sigmoid fits
    AB = [None] * len(svcs)
    if pl and cuda:
        # one launch for every fit: the kernel assembles each fit's decision values from the
        # batched decision partials through a position → partial-row map (negative codes: a
        # per-fold constant, −1 − code into consts; code −1 = 0.0 for positions no fold holds)
        E = ops.ext()
        pp = sol.get("platt_prep")
        if pp is None:      # (every Platt fold degenerate: nothing was prepared ahead)
            pp = platt_prep({id(p): sol[("hoff", id(p))] for p in all_probs if ("hoff", id(p)) in sol})
        src = sol.get("platt_src")
        srcmap, cdev, pdev, off = pp["srcmap"], pp["cdev"], pp["pdev"], pp["off"]
        dscr = torch.empty(off, dtype=torch.float64, device=device)   # (fits past 16k points)
        ABt = torch.empty(2 * len(pl), dtype=torch.float64, device=device)
        dmark("svc_platt_in")
        part_p, S, rowk_p, rho_p = ((src["part"].data_ptr(), src["S"], src["rowk"].data_ptr(), src["rho"].data_ptr())
                                    if src is not None else (0, 0, 0, 0))   # (every fold degenerate)
        # (PLATT_COOP: every fit's points over 8 workgroups meeting at a counter per Newton pass)
        cbar = torch.zeros(len(pl), dtype=torch.int32, device=device) if PLATT_COOP else None
        cpart = torch.empty(len(pl) * 2 * 8 * 6, dtype=torch.float64, device=device) if PLATT_COOP else None
        E.platt_batch(pdev.data_ptr(), len(pl), part_p, S, rowk_p, rho_p, cdev.data_ptr(), srcmap.data_ptr(),
                      dscr.data_ptr(), ABt.data_ptr(), cbar.data_ptr() if PLATT_COOP else 0,
                      cpart.data_ptr() if PLATT_COOP else 0, ops.stream_ptr(device))
        dmark("svc_platt")
        # the pairs' read-back queued right behind the Platt kernel (pinned, with an event): the host
        # waits for the Platt fits only, not for whatever is enqueued on this stream after them
        ab_host, ab_ev = stage(ABt)
        return dict(svcs=svcs, Zs=Zs, meta=meta, all_probs=all_probs, sol=sol, pl=pl, AB=AB, ABt=ABt,
                    ab_host=(ab_host, ab_ev),
                    keep=(pdev, srcmap, cdev, dscr, cbar, cpart), device=device, args=args, solver=solver, gamma_dev=gdev)
    for f in pl:
        svc, Z, mt = svcs[f], Zs[f], meta[f]
        l = mt["l"]
        dec = torch.zeros(l, dtype=torch.float64)
        from ..ops import reference as ref
        for p in (q for q in all_probs if q.fit == f and q.fold >= 0):
            if p.rows is None:
                dec[torch.as_tensor(p.held)] = p.const
                continue
            a, r, _ = sol[id(p)]
            yint = torch.where(torch.arange(a.numel()) < p.npos, 1.0, -1.0).to(torch.float64)
            Zh = Z[torch.as_tensor(p.held_rows, device=Z.device)].double()
            Zr = Z[torch.as_tensor(p.rows, device=Z.device)].double()
            d = ref.rbf_decision(Zh, Zr, (yint * a.cpu()).to(Zh.device), p.gamma, 0.0) - r
            dec[torch.as_tensor(p.held)] = -d.cpu()
        lab = np.where(np.arange(l) < mt["n0"], 1.0, -1.0)
        AB[f] = _sigmoid_train_host(dec.numpy(), lab)
    return dict(svcs=svcs, Zs=Zs, meta=meta, all_probs=all_probs, sol=sol, pl=pl, AB=AB, ABt=None,
                device=device, args=args, solver=solver)


def enqueue_svc_oof(st: dict, items, meta: torch.Tensor, col: int) -> bool:
    """Out-of-fold P(class 1) of fits launched by :func:`launch_svc_batch`, enqueued on the current
    stream behind their SMO and Platt kernels with no host synchronisation: ``items`` = [(fit f,
    scaled rows Zt [h, F] on the device, their row indices in ``meta`` (int64, device))]; fit f's
    final model's probability of each row is written to ``meta[rows, col]`` (one batched decision
    launch + one sigmoid/coupling launch).  Returns False when the batch has no device decision
    state (host solve, low-rank path, a degenerate problem): the caller then predicts as usual.
    Stale if :func:`finish_svc_batch` re-solves the batch (``st["resolved"]``)."""
    from .. import ops
    sol = st.get("sol")
    if st.get("done") or st.get("ABt") is None or sol is None or "_dec" not in sol or not items:
        return False
    dec_state, all_probs, pl, device = sol["_dec"], st["all_probs"], st["pl"], st["device"]
    finals = []
    for f, Zt, _ in items:
        p = [q for q in all_probs if q.fit == f and q.fold < 0][0]
        if p.rows is None or f not in pl or int(Zt.shape[1]) != dec_state["F"]:
            return False
        finals.append(p)
    E = ops.ext()
    s = ops.stream_ptr(device)
    per = 1024
    max_l = max(p.l for p in finals)
    S = (max_l + per - 1) // per
    dt = np.zeros(len(items), _DEC_DT)
    hoff = 0
    hs = []
    for i, ((f, Zt, _), p) in enumerate(zip(items, finals)):
        h = int(Zt.shape[0])
        dt[i] = (dec_state["zoff"][id(p)], hoff, p.l, h, -p.gamma * 1.4426950408889634, per)
        hoff += h
        hs.append(h)
    pre = sol.get("oof_pre")
    if pre is not None and pre["ids"] == [(f, id(Zt)) for f, Zt, _ in items] and pre["hoff"] == hoff:
        # the decisions came with the Platt launch (launch_svc_batch oof_items): only the sigmoid
        dec = pre["part"][pre["hoff0"]:pre["hoff0"] + hoff].to(torch.float64).sum(1).contiguous()
        return _svc_oof_tail(st, items, finals, dec, hs, meta, col, device, None, (pre,))
    hcat = torch.cat([Zt.to(torch.float32) for _, Zt, _ in items]).contiguous()
    part = torch.zeros(hoff, S, dtype=torch.float32, device=device)
    ddev = _dev_struct(dt, device)
    if st.get("gamma_dev") is not None:
        st["gamma_dev"].patch(ddev, _DEC_DT, "ngl2e", [f for f, _, _ in items])
    deps = sol.get("_deps")
    coef, rho_src = dec_state["coef"], None
    if deps is not None:
        # split join: wait for the groups of these final problems only, then y·α and ρ from them
        cur = torch.cuda.current_stream(device)
        ks = [dec_state["kof"][id(p)] for p in finals]
        deps["wait"](cur, ks)
        coef = (dec_state["sign"] * dec_state["alpha"].to(torch.float32)).contiguous()
        rho_src = deps["rho_for"](cur, ks)
    zsv, csv, cnt = _sv_compact(E, dec_state["zcat"], coef, dec_state["F"], ddev, len(items), device, s)
    E.svm_dec_batch(zsv.data_ptr(), csv.data_ptr(), hcat.data_ptr(), dec_state["F"],
                    ddev.data_ptr(), len(items), int(max(hs)), S, part.data_ptr(),
                    cnt.data_ptr() if cnt is not None else 0, s)
    dec = part.to(torch.float64).sum(1).contiguous()
    return _svc_oof_tail(st, items, finals, dec, hs, meta, col, device,
                         rho_src.index_select(0, _to_dev(np.asarray(ks, dtype=np.int64), device)).contiguous()
                         if rho_src is not None else None, (hcat, part, ddev, coef, zsv, csv, cnt))


# the decision launches read only each problem's support vectors (svm_sv_compact: ≈ 45 % of the
# points on the bench's problems; the skipped terms are exact zeros, the f32 partials group
# differently)
DEC_COMPACT = os.environ.get("HFENS_SVC_DEC_COMPACT", "1") != "0"
# the Platt sigmoid fits with each fit's points over 8 workgroups (svm.hip platt_coop_kernel)
PLATT_COOP = os.environ.get("HFENS_PLATT_COOP", "1") != "0"
# finish_svc_batch: the final models' set_fitted before the Platt pairs are read back (their
# bookkeeping overlaps the decision / Platt kernels; SVC.set_platt installs the pair after)
SET_BEFORE_PLATT = os.environ.get("HFENS_SVC_SET_BEFORE_PLATT", "1") != "0"


def _sv_compact(E, zcat, coef, F, ddev, P, device, s):
    """(rows, coefficients, per-problem counts) for a decision launch: the support vectors of every
    decision problem compacted in place of its points (same offsets), or the inputs unchanged."""
    if not DEC_COMPACT:
        return zcat, coef, None
    zc = torch.empty_like(zcat)
    cc = torch.empty_like(coef)
    cnt = torch.empty(P, dtype=torch.int32, device=device)
    E.svm_sv_compact(zcat.data_ptr(), coef.data_ptr(), F, ddev.data_ptr(), P, zc.data_ptr(), cc.data_ptr(),
                     cnt.data_ptr(), s)
    return zc, cc, cnt


def _svc_oof_tail(st, items, finals, dec, hs, meta, col, device, rho, keep) -> bool:
    """The out-of-fold probabilities from the decision values ``dec`` (rows of ``items`` in order):
    Platt sigmoid + coupling with each final model's ρ and (A, B), scattered into ``meta[:, col]``."""
    from .. import ops
    E = ops.ext()
    s = ops.stream_ptr(device)
    pl = st["pl"]
    hoff = int(dec.shape[0])
    model = torch.repeat_interleave(torch.arange(len(items), dtype=torch.int32),
                                    torch.as_tensor(hs, dtype=torch.int64))
    model = _to_dev(model.numpy(), device)
    if rho is None:
        rho = torch.stack([st["sol"][id(p)][1].reshape(()).to(torch.float64) for p in finals]).contiguous()
    sel = _to_dev(np.array([pl.index(f) for f, _, _ in items], dtype=np.int64), device)
    AB = st["ABt"].view(-1, 2).index_select(0, sel).reshape(-1).contiguous()
    rows = torch.cat([r.to(torch.int64) for _, _, r in items]).contiguous()
    assert meta.dtype == torch.float64 and meta.is_contiguous() and meta.dim() == 2
    E.svc_oof(dec.data_ptr(), model.data_ptr(), rho.data_ptr(), AB.data_ptr(), rows.data_ptr(), meta.data_ptr(),
              int(meta.shape[1]), int(col), hoff, s)
    from ..utils.timing import dmark
    dmark("svc_oof")
    st["oof_keep"] = keep + (dec, model, rho, sel, AB, rows)
    return True


def finish_svc_batch(st: dict, defer=None):
    """Platt parameters to the host, support-vector extraction, ``set_fitted``.  ``defer``: fits
    whose ``set_fitted`` (≈ 0.3 ms of host work each) is left to the closure ``st["finish_rest"]``
    (the stacking trainer: the fold models, when the device already computed their out-of-fold
    column, are not needed at all)."""
    if st.get("done"):
        return st["svcs"]
    svcs, Zs, meta, all_probs, sol, AB, device = (st["svcs"], st["Zs"], st["meta"], st["all_probs"],
                                                   st["sol"], st["AB"], st["device"])
    if sol.get("_deps") is not None:
        # (split join) everything from here on sees the whole batch: the refit's final problem too
        torch.cuda.current_stream(device).wait_event(sol["_deps"]["join_ev"])
    early = sol.get("_early")
    finals = [[q for q in all_probs if q.fit == f and q.fold < 0][0] for f in range(len(svcs))]
    if early is not None and early["ids"] != [id(p) for p in finals]:
        early = None
    from ..utils.timing import hmark
    if early is not None:
        hmark("svc_early_wait")
        host_e = landed(early["host"], early["ev"])
        hmark("svc_early_synced")
        smo_failed = early["has_err"] and host_e[-1] != 0.0
    else:
        err = sol.get("smo_err")
        smo_failed = err is not None and float(err.max()) != 0.0
    if st.get("gamma_dev") is not None:
        st["gamma_dev"].resolve(all_probs, meta)     # (the host's γ; raises on non-finite scaled rows)
        st["gamma_dev"] = None
    if smo_failed:
        # cooperative SMO: a member exchange timed out (members not co-resident beside concurrent
        # work) → re-solve with the one-workgroup kernel; working-set SMO: a problem needed more
        # than WS_ROUNDS_AHEAD rounds → re-solve with host-checked rounds.  Under a process group
        # err is part of the all-reduced solution vector, so every rank takes this branch together.
        if st.get("retried"):
            raise RuntimeError("SMO: the synchronous re-solve failed again")
        import warnings
        ws = st.get("solver") == "ws"
        warnings.warn("working-set SMO needed more than the rounds enqueued ahead; re-solving with host-checked rounds"
                      if ws else
                      "cooperative SMO timed out waiting for a member; re-solving with one workgroup per problem")
        flag = _WS_SYNC if ws else _FORCE_SINGLE
        flag[0] = True
        st["resolved"] = True   # (anything enqueued from the first solution, e.g. a device OOF, is stale)
        try:
            st2 = launch_svc_batch(*st["args"])
        finally:
            flag[0] = False
        st2["retried"] = True
        LAST_SMO_INFO["ws_resolve" if ws else "coop_fallback"] = True
        return finish_svc_batch(st2)   # (no deferral after a re-solve: everything is final here)
    # ---- final models: ONE device→host read of the Platt (A, B) pairs and every final solve's
    # support mask, ρ and iteration count; the bookkeeping is then numpy, the gathers non-blocking
    # ---- final models: the support masks, ρ and iteration counts of every final solve (the early
    # read, or one read with the Platt pairs); the bookkeeping is then numpy, the gathers non-blocking
    sols = [sol[id(p)] for p in finals]
    ls = [int(a.numel()) for a, _, _ in sols]
    from ..utils.timing import hmark
    if early is not None:
        host = host_e
    else:
        host = torch.cat([torch.cat([(a > 0).to(torch.float64).reshape(-1) for a, _, _ in sols]),
                          torch.stack([torch.as_tensor(r).to(device=device, dtype=torch.float64).reshape(()) for _, r, _ in sols]),
                          torch.stack([torch.as_tensor(it).to(device=device, dtype=torch.float64).reshape(()) for _, _, it in sols])]
                         + ([st["ABt"].to(device=device, dtype=torch.float64)] if st["ABt"] is not None else [])
                         ).cpu().numpy()
    hmark("svc_host_read")
    nl = sum(ls)
    offs = np.concatenate([[0], np.cumsum(ls)])

    def prep_one(f):
        """Everything of fit f's set_fitted but the Platt pair (device gathers enqueued)."""
        svc, Z, mt = svcs[f], Zs[f], meta[f]
        a = sols[f][0].to(device)
        pos_np = np.nonzero(host[offs[f]:offs[f + 1]] > 0.5)[0]
        pos_idx = _to_dev(pos_np.astype(np.int64), device)
        yint = torch.where(pos_idx < mt["n0"], 1.0, -1.0).to(torch.float64)
        coef = yint * a[pos_idx]
        support = _to_dev(mt["grouped"][pos_np].astype(np.int64), device)
        n_sv0 = int((pos_np < mt["n0"]).sum())
        return dict(support=support, support_vectors=Z[support].to(torch.float64),
                    n_support=[n_sv0, int(pos_np.shape[0]) - n_sv0], dual_coef_libsvm=coef,
                    rho=float(host[nl + f]), gamma=mt["gamma"],
                    class_weight=torch.tensor([mt["C0"] / svc.C, mt["C1"] / svc.C]),
                    shape_fit=tuple(Z.shape), n_features=Z.shape[1], device=device)

    def set_one(f, kw, platt=True):
        A, B = AB[f] if platt and AB[f] is not None else (0.0, 0.0)
        svcs[f].set_fitted(probA=A, probB=B, **kw)
        svcs[f].n_iter_ = int(host[nl + len(svcs) + f])

    def read_ab():
        if st["ABt"] is None:
            return
        if early is not None and st.get("ab_host") is not None:
            ABc = landed(*st["ab_host"])
        elif early is not None:
            ABc = st["ABt"].to(torch.float64).cpu().numpy()
        else:
            ABc = host[nl + 2 * len(svcs):]
        if not np.isfinite(ABc).all():
            from ..utils.guards import NonFiniteError
            raise NonFiniteError(f"SVC Platt sigmoid (A, B): {int((~np.isfinite(ABc)).sum())} non-finite value(s)")
        for k, f in enumerate(st["pl"]):
            AB[f] = (float(ABc[2 * k]), float(ABc[2 * k + 1]))

    def fit_one(f):
        set_one(f, prep_one(f))

    later = [f for f in range(len(svcs)) if defer is not None and f in defer]
    now = [f for f in range(len(svcs)) if f not in later]
    kws = {f: prep_one(f) for f in now}     # (with the early read: while the Platt kernels run)
    pre = SET_BEFORE_PLATT and early is not None and st.get("ab_host") is not None and st["ABt"] is not None
    if pre:
        # set_fitted too while the Platt kernels run; the pair (device: the kernel's own output)
        # goes in after its read-back
        for f in now:
            set_one(f, kws[f], platt=False)
    read_ab()
    hmark("svc_platt_read")
    if pre:
        slot = {f: k for k, f in enumerate(st["pl"])}
        for f in now:
            A, B = AB[f] if AB[f] is not None else (0.0, 0.0)
            k = slot.get(f)
            svcs[f].set_platt(A, B, st["ABt"][2 * k:2 * k + 2] if k is not None else None)
    else:
        for f in now:
            set_one(f, kws[f])
    hmark("svc_set_fitted")
    if later:
        pending = list(later)

        def rest():
            # (no reference to st: a closure stored in st that refers back to it made a reference
            # cycle that kept the batch's device buffers — ≈ 77 MB per headline fit with the working-
            # set runs below — alive until a full GC, profiles/r6_runs/r6p)
            while pending:
                fit_one(pending.pop(0))
        st["finish_rest"] = rest
    return svcs

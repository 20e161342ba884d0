"""Host simulation of the working-set SMO (svm_ws.hip) on the bench's critical SVC problem:
outer rounds and inner pairs as a function of the working-set size q and the inner stop fraction.

Builds the headline's refit problem (10k rows × 40 → impute → LassoCV top-17 → StandardScaler,
γ = 1/17, balanced C) with scikit-learn on the CPU, then runs the same outer loop as the GPU
solver (q/4 most violating I_up + q/4 I_low points, previous round's new picks kept, libsvm WSS3
pairs inside B until the local gap < frac · the round's starting local gap, f64 global gap
< 1e-3 to stop).  Usage: python scripts/probes/ws_qsim.py [rows] [q ...]
"""
import os
import sys
import time

import numpy as np


def build_problem(rows=10000, seed=2020):
    sys.path.insert(0, ".")
    from hfens.io.synth import make_hf_cohort
    from sklearn.impute import KNNImputer
    from sklearn.linear_model import LassoCV
    from sklearn.feature_selection import SelectFromModel
    X, y, _ = make_hf_cohort(rows, 40, seed=seed, nan_frac=0.02)
    X = KNNImputer(n_neighbors=1).fit_transform(X)
    sfm = SelectFromModel(LassoCV(cv=10, random_state=2020), threshold=-np.inf, max_features=17).fit(X, y)
    Z = X[:, sfm.get_support()]
    Z = (Z - Z.mean(0)) / np.where(Z.std(0) > 0, Z.std(0), 1.0)
    F = Z.shape[1]
    gamma = 1.0 / (F * Z.var())
    n1 = (y == 1).sum()
    n0 = len(y) - n1
    cw = len(y) / (2.0 * np.array([n0, n1]))
    # libsvm's internal +1 is the first label seen; the framework groups class 0 as +1
    order = np.concatenate([np.flatnonzero(y == 0), np.flatnonzero(y == 1)])
    Z = Z[order]
    yv = np.where(np.arange(len(y)) < n0, 1.0, -1.0)
    C = np.where(yv > 0, cw[0], cw[1])
    return KernelCols(Z.astype(np.float32), gamma), yv, C


class KernelCols:
    """K[:, cols] / K[np.ix_(B, B)] of the RBF kernel computed on demand (no l² matrix)."""

    def __init__(self, Z, gamma):
        self.Z, self.gamma = Z, gamma
        self.sq = (Z.astype(np.float64) ** 2).sum(1)

    def block(self, rows, cols):
        Zr, Zc = self.Z[rows].astype(np.float64), self.Z[cols].astype(np.float64)
        d = self.sq[rows][:, None] + self.sq[cols][None, :] - 2.0 * Zr @ Zc.T
        return np.exp(-self.gamma * np.maximum(d, 0.0)).astype(np.float32)


def smo_sub(KB, GB, aB, CB, yB, tol, max_inner):
    """libsvm WSS3 pairs on the working set (in place); returns the pair count."""
    n = 0
    while n < max_inner:
        up = np.where(yB > 0, aB < CB, aB > 0)
        low = np.where(yB > 0, aB > 0, aB < CB)
        if not up.any() or not low.any():
            break
        f = -yB * GB
        fu = np.where(up, f, -np.inf)
        i = int(np.argmax(fu))
        gmax = fu[i]
        fl = np.where(low, f, np.inf)
        if gmax - fl.min() < tol:
            break
        gd = gmax - f                       # = Gmax + yG for low points
        quad = np.maximum(2.0 - 2.0 * KB[i], 1e-12)
        obj = np.where(low & (gd > 0), gd * gd / quad, -np.inf)
        j = int(np.argmax(obj))
        if obj[j] == -np.inf:
            break
        yi, yj = yB[i], yB[j]
        Ci, Cj = CB[i], CB[j]
        ai, aj = aB[i], aB[j]
        q = max(2.0 - 2.0 * KB[i, j], 1e-12)
        if yi != yj:
            delta = (-GB[i] - GB[j]) / q
            diff = ai - aj
            ai += delta
            aj += delta
            if diff > 0:
                if aj < 0:
                    aj, ai = 0.0, diff
            elif ai < 0:
                ai, aj = 0.0, -diff
            if diff > Ci - Cj:
                if ai > Ci:
                    ai, aj = Ci, Ci - diff
            elif aj > Cj:
                aj, ai = Cj, Cj + diff
        else:
            delta = (GB[i] - GB[j]) / q
            s = ai + aj
            ai -= delta
            aj += delta
            if s > Ci:
                if ai > Ci:
                    ai, aj = Ci, s - Ci
            elif aj < 0:
                aj, ai = 0.0, s
            if s > Cj:
                if aj > Cj:
                    aj, ai = Cj, s - Cj
            elif ai < 0:
                ai, aj = 0.0, s
        dai, daj = ai - aB[i], aj - aB[j]
        GB += yB * (KB[i] * (yi * dai) + KB[j] * (yj * daj))
        aB[i], aB[j] = ai, aj
        n += 1
    return n


def ws(K, yv, C, q, frac, eps=1e-3, max_inner=None, reuse=True):
    l = len(yv)
    max_inner = max_inner or 8 * q
    a = np.zeros(l)
    G = -np.ones(l)
    outer = inner = 0
    prev = np.array([], dtype=int)
    nchanged = []
    while True:
        up = np.where(yv > 0, a < C, a > 0)
        low = np.where(yv > 0, a > 0, a < C)
        f = -yv * G
        gap = f[up].max() - f[low].min()
        if gap < eps or outer > 5000:
            break
        iu = np.flatnonzero(up)
        il = np.flatnonzero(low)
        su = iu[np.argsort(-f[iu], kind="stable")[: min(q // 4, len(iu))]]
        il2 = il[~np.isin(il, su)]
        sl = il2[np.argsort(f[il2], kind="stable")[: min(q // 4, len(il2))]]
        new = np.concatenate([np.sort(su), np.sort(sl)])
        keep = prev[~np.isin(prev, new)] if reuse else np.array([], dtype=int)
        B = np.concatenate([new, keep])[:q]
        prev = new
        KB = K.block(B, B).astype(np.float64)
        aB = a[B].copy()
        GB = G[B].copy()
        yB = yv[B]
        upB = np.where(yB > 0, aB < C[B], aB > 0)
        lowB = np.where(yB > 0, aB > 0, aB < C[B])
        fb = -yB * GB
        gap0 = fb[upB].max() - fb[lowB].min()
        n_in = smo_sub(KB, GB, aB, C[B], yB, max(eps, frac * gap0), max_inner)
        inner += n_in
        da = aB - a[B]
        ch = np.flatnonzero(da != 0)
        nchanged.append(len(ch))
        G += yv * (K.block(np.arange(l), B[ch]).astype(np.float64) @ (yB[ch] * da[ch]))
        a[B] = aB
        outer += 1
        if n_in == 0:
            break
    nsv = int((a > 0).sum())
    sv = np.flatnonzero(a > 0)
    obj = 0.5 * (a[sv] * yv[sv]) @ (K.block(sv, sv).astype(np.float64) @ (a[sv] * yv[sv])) - a.sum() if len(sv) <= 20000 else float("nan")
    return dict(q=q, frac=frac, rounds=outer, pairs=inner, gap=float(gap), nsv=nsv,
                changed_mean=float(np.mean(nchanged)) if nchanged else 0.0, obj=float(obj))


if __name__ == "__main__":
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    qs = [int(v) for v in sys.argv[2:]] or [1024, 512, 256, 128]
    t = time.time()
    K, yv, C = build_problem(rows)
    print(f"problem: l={len(yv)} npos={(yv > 0).sum()} C={C[0]:.4f}/{C[-1]:.4f} ({time.time() - t:.1f}s)", flush=True)
    fracs = [float(v) for v in os.environ.get("FRACS", "0.1,0.2,0.4").split(",")]
    for q in qs:
        for frac in fracs:
            t = time.time()
            r = ws(K, yv, C, q, frac)
            print(r, f"{time.time() - t:.1f}s", flush=True)

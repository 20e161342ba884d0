"""Would two SMO pairs per inner iteration shorten the critical problem's pair loop?

The q = 1024 inner solver (svm_ws.hip ws_solve_kernel) is latency-bound: one pair = two block
reductions + two dependent kernel rows (≈ 3.46k cycles, bench diag ``ws_critical``).  A second,
independent pair picked in the SAME reductions (i2 = the runner-up I_up point, or the best I_up
point of the other slot half; j2 = its WSS3 partner) would ride in the same barriers, its two rows
computed beside the first pair's; its step is taken with the gradient already corrected for the
first pair (an exact two-variable minimisation, so the dual still decreases monotonically).  Worth
it only if the extra pairs it needs are few: this host simulation counts pairs and inner
iterations (= the dependent-chain length) for the bench's 10k refit problem, cold and from the
cascade seed the solver uses (parts at eps 0.3, q = 512, 8 rounds; then q = 1024, frac 0.2).
Usage: python scripts/probes/ws_pair2_sim.py [rows]

Result (round 6): host simulation "half" mode — 4413 → 4425 pairs in 2718 instead of 4413 main
iterations (parts: 667 vs 1158).  Built on the GPU (ws_solve_kernel with a second pair,
profiles/r6_runs/r6af): 5205 pairs (+6 %) but the same inner cycles as one pair per iteration
(21.2 M vs 21.3 M s_memtime cycles on the critical problem) — a pair iteration is bound by its
per-slot VALU work (two kernel rows, two key passes), which the second pair doubles; only the
barriers are shared.  The one-pair kernel also lost 26 % (3457 → 4354 cycles / pair) to the
runtime two-pair branches.  Reverted.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, "scripts/probes")
import ws_qsim  # noqa: E402
from ws_cascade_sim import parts_of  # noqa: E402


def two_var_step(ai, aj, Gi, Gj, yi, yj, Ci, Cj, Kij):
    q = max(2.0 - 2.0 * Kij, 1e-12)
    if yi != yj:
        delta = (-Gi - Gj) / q
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
        delta = (Gi - Gj) / q
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
    return ai, aj


def smo_sub_multi(KB, GB, aB, CB, yB, tol, max_inner, mode, stats):
    """WSS3 pairs on B; mode "one" = libsvm's rule, "top2" / "half" = a second pair per iteration."""
    n = 0
    half = np.arange(len(yB)) % 2
    while n < max_inner:
        up = np.where(yB > 0, aB < CB, aB > 0)
        low = np.where(yB > 0, aB > 0, aB < CB)
        if not up.any() or not low.any():
            break
        f = -yB * GB
        fu = np.where(up, f, -np.inf)
        i1 = int(np.argmax(fu))
        gmax = fu[i1]
        fl = np.where(low, f, np.inf)
        if gmax - fl.min() < tol:
            break

        def partner(i):
            gd = f[i] - f
            quad = np.maximum(2.0 - 2.0 * KB[i], 1e-12)
            obj = np.where(low & (gd > 0), gd * gd / quad, -np.inf)
            j = int(np.argmax(obj))
            return j, obj[j] > -np.inf
        j1, ok1 = partner(i1)
        if not ok1:
            break
        second = False
        if mode != "one":
            fu2 = fu.copy()
            if mode == "top2":
                fu2[i1] = -np.inf
            else:
                fu2[half == half[i1]] = -np.inf
            i2 = int(np.argmax(fu2))
            if fu2[i2] > -np.inf:
                j2, ok2 = partner(i2)
                second = ok2 and j2 not in (i1, j1) and i2 != j1
        pairs = [(i1, j1)] + ([(i2, j2)] if second else [])
        for i, j in pairs:
            ai, aj = two_var_step(aB[i], aB[j], GB[i], GB[j], yB[i], yB[j], CB[i], CB[j], KB[i, j])
            dai, daj = ai - aB[i], aj - aB[j]
            GB += yB * (KB[i] * (yB[i] * dai) + KB[j] * (yB[j] * daj))
            aB[i], aB[j] = ai, aj
            n += 1
        stats["iters"] += 1
        stats["second"] += int(second)
    return n


def solve(K, yv, C, q, frac, a0, eps, mode, rows=None, max_rounds=5000):
    if rows is not None:
        Ks = ws_qsim.KernelCols(K.Z[rows], K.gamma)
        return solve(Ks, yv[rows], C[rows], q, frac, a0[rows] if a0 is not None else None, eps, mode,
                     max_rounds=max_rounds)
    l = len(yv)
    a = np.zeros(l) if a0 is None else a0.copy()
    G = -np.ones(l)
    sv = np.flatnonzero(a > 0)
    for s in range(0, l, 4096):
        blk = np.arange(s, min(l, s + 4096))
        if len(sv):
            G[blk] += yv[blk] * (K.block(blk, sv).astype(np.float64) @ (yv[sv] * a[sv]))
    st = dict(iters=0, second=0, rounds=0, pairs=0)
    prev = np.array([], dtype=int)
    while st["rounds"] < max_rounds:
        up = np.where(yv > 0, a < C, a > 0)
        low = np.where(yv > 0, a > 0, a < C)
        f = -yv * G
        gap = f[up].max() - f[low].min()
        if gap < eps:
            break
        iu, il = np.flatnonzero(up), np.flatnonzero(low)
        su = iu[np.argsort(-f[iu], kind="stable")[: min(q // 4, len(iu))]]
        il2 = il[~np.isin(il, su)]
        sl = il2[np.argsort(f[il2], kind="stable")[: min(q // 4, len(il2))]]
        new = np.concatenate([np.sort(su), np.sort(sl)])
        keep = prev[~np.isin(prev, new)]
        B = np.concatenate([new, keep])[:q]
        prev = new
        KB = K.block(B, B).astype(np.float64)
        aB, GB, yB = a[B].copy(), G[B].copy(), yv[B]
        upB = np.where(yB > 0, aB < C[B], aB > 0)
        lowB = np.where(yB > 0, aB > 0, aB < C[B])
        fb = -yB * GB
        gap0 = fb[upB].max() - fb[lowB].min()
        n_in = smo_sub_multi(KB, GB, aB, C[B], yB, max(eps, frac * gap0), 4096, mode, st)
        st["pairs"] += n_in
        da = aB - a[B]
        ch = np.flatnonzero(da != 0)
        if len(ch):
            G += yv * (K.block(np.arange(l), B[ch]).astype(np.float64) @ (yB[ch] * da[ch]))
        a[B] = aB
        st["rounds"] += 1
        if n_in == 0:
            break
    st["gap"] = float(gap)
    return a, st


if __name__ == "__main__":
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    t = time.time()
    K, yv, C = ws_qsim.build_problem(rows)
    print(f"problem l={len(yv)} ({time.time() - t:.1f}s)", flush=True)
    P = int(os.environ.get("PARTS", "4"))
    probe = np.random.default_rng(1).choice(len(yv), 1000, replace=False)

    def dec(a):
        sv = np.flatnonzero(a > 0)
        return K.block(probe, sv).astype(np.float64) @ (yv[sv] * a[sv])
    ref = None
    for mode in os.environ.get("MODES", "one,top2,half").split(","):
        a0 = np.zeros(len(yv))
        part = []
        for rws in parts_of(yv, P):
            ap, sp = solve(K, yv, C, 512, 0.2, None, 0.3, mode, rows=rws, max_rounds=8)
            a0[rws] = ap
            part.append(sp)
        a, st = solve(K, yv, C, 1024, 0.2, a0, 1e-3, mode)
        d = dec(a)
        ref = d if ref is None else ref
        print(f"{mode}: parts iters max {max(s['iters'] for s in part)} pairs max {max(s['pairs'] for s in part)} | "
              f"main {st} | critical iters {max(s['iters'] for s in part) + st['iters']} "
              f"max|Δdec| vs one {np.abs(d - ref).max():.3g}", flush=True)

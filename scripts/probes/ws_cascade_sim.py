"""Would a cascade seed cut the critical SVC problem's pair count?

The headline's 10k-point refit problem (scripts/probes/ws_qsim.py) is split into P disjoint,
class-stratified parts.  Each part is solved as its own SVC with the SAME per-class C (the
refit's balanced weights), so the concatenated part solutions satisfy the full problem's box and
equality constraints: a feasible warm start.  The full problem is then solved from that seed by the
same working-set rule.  Parts run side by side on separate CUs, so the critical pair count is
max(part pairs) + full-from-seed pairs (vs the cold full solve).  The seed's stopping tolerance
(SEED_EPS) can be looser than the final eps.  Usage: python scripts/probes/ws_cascade_sim.py [rows]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, "scripts/probes")
import ws_qsim  # noqa: E402


def ws_seeded(K, yv, C, q, frac, a0, eps=1e-3, rows=None):
    """ws_qsim.ws with α = a0 (G = Qα − 1 computed once) on the sub-problem `rows` (all if None)."""
    if rows is not None:
        Ks = ws_qsim.KernelCols(K.Z[rows], K.gamma)
        return ws_seeded(Ks, yv[rows], C[rows], q, frac, a0[rows] if a0 is not None else None, eps)
    l = len(yv)
    a = np.zeros(l) if a0 is None else a0.copy()
    G = -np.ones(l)
    sv = np.flatnonzero(a > 0)
    if len(sv):
        for s in range(0, l, 4096):
            blk = np.arange(s, min(l, s + 4096))
            G[blk] += yv[blk] * (K.block(blk, sv).astype(np.float64) @ (yv[sv] * a[sv]))
    outer = inner = 0
    prev = np.array([], dtype=int)
    while True:
        up = np.where(yv > 0, a < C, a > 0)
        low = np.where(yv > 0, a > 0, a < C)
        f = -yv * G
        gap = f[up].max() - f[low].min()
        if gap < eps or outer > 5000:
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
        n_in = ws_qsim.smo_sub(KB, GB, aB, C[B], yB, max(eps, frac * gap0), 8 * q)
        inner += n_in
        da = aB - a[B]
        ch = np.flatnonzero(da != 0)
        if len(ch):
            G += yv * (K.block(np.arange(l), B[ch]).astype(np.float64) @ (yB[ch] * da[ch]))
        a[B] = aB
        outer += 1
        if n_in == 0:
            break
    return a, dict(rounds=outer, pairs=inner, gap=float(gap), nsv=int((a > 0).sum()))


def parts_of(yv, P, seed=0):
    rng = np.random.default_rng(seed)
    lab = np.empty(len(yv), dtype=int)
    for cls in (1.0, -1.0):
        idx = np.flatnonzero(yv == cls)
        lab[idx] = rng.permutation(len(idx)) % P
    return [np.flatnonzero(lab == p) for p in range(P)]


if __name__ == "__main__":
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    q = int(os.environ.get("Q", "1024"))
    frac = float(os.environ.get("FRAC", "0.2"))
    t = time.time()
    K, yv, C = ws_qsim.build_problem(rows)
    print(f"problem l={len(yv)} ({time.time() - t:.1f}s)", flush=True)
    a_cold, r_cold = ws_seeded(K, yv, C, q, frac, None)
    print("cold", r_cold, flush=True)
    probe = np.random.default_rng(1).choice(len(yv), 1000, replace=False)

    def dec(a):
        sv = np.flatnonzero(a > 0)
        return K.block(probe, sv).astype(np.float64) @ (yv[sv] * a[sv])
    d_cold = dec(a_cold)
    a_q512, r_q512 = ws_seeded(K, yv, C, q // 2, frac, None)
    print(f"cold q/2 {r_q512} natural max|Δdec| {np.abs(dec(a_q512) - d_cold).max():.3g}", flush=True)
    for P in [int(v) for v in os.environ.get("PARTS", "2,4,8").split(",")]:
        for seps in [float(v) for v in os.environ.get("SEED_EPS", "1e-3,1e-2").split(",")]:
            a0 = np.zeros(len(yv))
            part_pairs = []
            for rws in parts_of(yv, P):
                qp = min(q, 1 << int(np.ceil(np.log2(max(64, len(rws) // 4)))))
                ap, rp = ws_seeded(K, yv, C, qp, frac, None, seps, rows=rws)
                a0[rws] = ap
                part_pairs.append(rp["pairs"])
            assert abs((yv * a0).sum()) < 1e-6 * len(yv) and (a0 <= C + 1e-12).all()
            a_s, r_s = ws_seeded(K, yv, C, q, frac, a0)
            da = np.abs(a_s - a_cold).max()
            print(f"P={P} seed_eps={seps:g} part_pairs max={max(part_pairs)} {part_pairs} "
                  f"full_from_seed={r_s} critical={max(part_pairs) + r_s['pairs']} "
                  f"vs cold {r_cold['pairs']}  max|Δα|={da:.3g} max|Δdec|={np.abs(dec(a_s) - d_cold).max():.3g}", flush=True)

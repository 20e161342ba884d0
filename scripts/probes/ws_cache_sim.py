"""How often would a small kernel-row cache hit inside the working-set SMO's pair loop?

Runs the host simulation of svm_ws.hip (scripts/probes/ws_qsim.py: the headline's 10k-point refit
problem, q = 1024, inner stop fraction 0.2) and records every pair's (i, j) slot picks; reports the
share of row lookups (i then j per pair) that an LRU cache of k rows, kept across the pairs of one
working-set round, would serve.  Usage: python scripts/probes/ws_cache_sim.py [rows]
"""
import collections
import sys

import numpy as np

sys.path.insert(0, "scripts/probes")
import ws_qsim  # noqa: E402

PICKS = []
_orig = ws_qsim.smo_sub


def smo_sub_rec(KB, GB, aB, CB, yB, tol, max_inner):
    picks = []
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
        gd = gmax - f
        quad = np.maximum(2.0 - 2.0 * KB[i], 1e-12)
        obj = np.where(low & (gd > 0), gd * gd / quad, -np.inf)
        j = int(np.argmax(obj))
        if obj[j] == -np.inf:
            break
        picks.append((i, j))
        # one pair of the real rule (ws_qsim.smo_sub with max_inner = 1 applies exactly this step)
        _orig(KB, GB, aB, CB, yB, -1.0, 1)
        n += 1
    PICKS.append(picks)
    return n


ws_qsim.smo_sub = smo_sub_rec


def lru_hits(picks, k):
    hits = tot = 0
    for rnd in picks:
        cache = collections.OrderedDict()
        for i, j in rnd:
            for r in (i, j):
                tot += 1
                if r in cache:
                    hits += 1
                    cache.move_to_end(r)
                else:
                    cache[r] = True
                    if len(cache) > k:
                        cache.popitem(last=False)
    return hits / max(tot, 1), tot


if __name__ == "__main__":
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    K, yv, C = ws_qsim.build_problem(rows)
    r = ws_qsim.ws(K, yv, C, 1024, 0.2)
    print(r)
    npairs = sum(len(p) for p in PICKS)
    print("pairs", npairs, "rounds", len(PICKS))
    for k in (1, 2, 4, 8, 12, 16, 32, 64):
        h, tot = lru_hits(PICKS, k)
        print(f"LRU {k:3d} rows: hit {h:.3f} of {tot} lookups")
    # i repeats the previous pair's i / j
    same_i = sum(1 for p in PICKS for a, b in zip(p, p[1:]) if b[0] in a)
    print("i in previous pair:", same_i / max(1, npairs - len(PICKS)))

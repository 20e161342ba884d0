"""Two-level cascade seed for the headline 10k problem (host simulation, ws_cascade_sim.py
machinery): level-1 parts, then merged part groups solved from their seed, then the full problem.
Round 6 record: profiles/r6_runs/cascade_two_level_sim.log (no gain over one level)."""
import os, sys, time
import numpy as np
sys.path.insert(0, "scripts/probes")
import ws_qsim
from ws_cascade_sim import ws_seeded, parts_of
K, yv, C = ws_qsim.build_problem(10000)
q, frac = 1024, 0.2
t=time.time()
a_cold, r_cold = ws_seeded(K, yv, C, q, frac, None)
print("cold", r_cold, round(time.time()-t,1), flush=True)
def level(a0, groups, eps, qmax=1024):
    a = a0.copy(); stats=[]
    for rws in groups:
        qp = min(qmax, 1 << int(np.ceil(np.log2(max(64, len(rws) // 4)))))
        ap, rp = ws_seeded(K, yv, C, qp, frac, a, eps, rows=rws)
        a[rws] = ap; stats.append((rp["rounds"], rp["pairs"]))
    return a, stats
def cost(st):  # critical (rounds, pairs) of a level: max over groups
    return max(s[0] for s in st), max(s[1] for s in st)
P1 = parts_of(yv, 8)
for e1 in (0.1, 0.03):
    a1, s1 = level(np.zeros(len(yv)), P1, e1, 512)
    af, rf = ws_seeded(K, yv, C, q, frac, a1)
    print(f"1-level e1={e1}: L1 {cost(s1)} final ({rf['rounds']},{rf['pairs']})", flush=True)
    for merge, e2 in ((2, 0.03), (2, 0.01), (4, 0.03)):
        groups = [np.concatenate([P1[j] for j in range(8) if j % merge == g]) for g in range(merge)]
        a2, s2 = level(a1, groups, e2)
        af2, rf2 = ws_seeded(K, yv, C, q, frac, a2)
        print(f"2-level e1={e1} merge->{merge} e2={e2}: L1 {cost(s1)} L2 {cost(s2)} final ({rf2['rounds']},{rf2['pairs']})", flush=True)

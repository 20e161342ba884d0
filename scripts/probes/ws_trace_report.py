"""Per-round durations of the working-set SMO kernels (ws_select / ws_solve / ws_gupdate) in the
last develop() of a kernel trace, and the logistic-regression kernels' durations."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
sel = [i for i, k in enumerate(ks) if "ws_select_kernel" in k[2]]
# the last fit: its rounds are the last run of consecutive select launches (64 per fit)
last = sel[-64:]
t0 = ks[last[0]][0]
span = [k for k in ks[last[0]:] if k[0] >= t0]
solve = [(s, e) for s, e, n in span if "ws_solve_kernel" in n][:64]
selk = [(s, e) for s, e, n in span if "ws_select_kernel" in n][:64]
upd = [(s, e) for s, e, n in span if "ws_gupdate_kernel" in n][:64]
print("round  select_us  solve_us  gupdate_us  round_wall_us")
for r in range(len(solve)):
    a = selk[r][1] - selk[r][0]
    b = solve[r][1] - solve[r][0]
    c = upd[r][1] - upd[r][0] if r < len(upd) else 0
    w = (upd[r][1] if r < len(upd) else solve[r][1]) - selk[r][0]
    if r < 40 or b > 5000:
        print(f"{r:5d} {a / 1e3:10.1f} {b / 1e3:9.1f} {c / 1e3:11.1f} {w / 1e3:14.1f}")
print("sum solve ms", sum(e - s for s, e in solve) / 1e6, "sum select ms", sum(e - s for s, e in selk) / 1e6,
      "sum gupdate ms", sum(e - s for s, e in upd) / 1e6,
      "rounds wall ms", (upd[-1][1] - selk[0][0]) / 1e6 if upd else 0)
lr = [(e - s) / 1e6 for s, e, n in ks if "logreg_fused_kernel" in n]
print("logreg kernels ms (all fits):", [round(x, 2) for x in lr[-6:]])

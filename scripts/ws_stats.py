"""Headline fit with the base models run one after another (HFENS_CONCURRENT_BASES=0 set by the
caller): device-synchronised stage times per base model, plus the working-set SMO's per-problem
rounds, pairs and in-kernel phase cycles (svm_ws.hip s_memtime stamps)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
for rep in range(4):
    tm = StageTimer(enabled=True, device=dev)
    develop(Xd, yd, Xs, ys, names, device=dev, evaluate=False, timer=tm)
torch.cuda.synchronize()
print(tm.table())
st = smo.LAST_WS_STATS
if smo.LAST_CASCADE.get("stats"):
    cs = smo.LAST_CASCADE["stats"]()
    print("cascade parts", smo.LAST_CASCADE["parts"], "outer max", int(cs["outer"].max()), "mean",
          float(cs["outer"].mean()), "inner max", int(cs["inner"].max()), "gap max", float(cs["gap"].max()))
print("q", st.get("q"), "outer", st["outer"].tolist())
print("inner", st["inner"].tolist())
clk = 2.4e3  # cycles per µs (s_memtime ≈ shader clock)
for k in np.argsort(-st["inner"])[:4]:
    o, i = int(st["outer"][k]), int(st["inner"][k])
    print(f"problem {k}: outer {o} inner {i}  select {st['cyc_select'][k] / clk / max(o, 1):.1f} µs/round  "
          f"build {st['cyc_build'][k] / clk / max(o, 1):.1f} µs/round  inner {st['cyc_inner'][k] / clk / max(i, 1):.3f} µs/pair "
          f"({st['cyc_inner'][k] / clk / 1e3:.2f} ms)")
ph = st.get("phases")
if ph is not None:
    names = (["keys+i max", "fetch i+row_i", "j keys+max", "fetch j+row_j+step", "update", "-"]
             if st.get("q") == 256 else ["keys", "barrier1+i", "row_i", "barrier2+j", "pair", "row_j+grad"])
    k = int(np.argmax(st["inner"]))
    tot = ph[k].sum()
    print("phases of problem", k, "(cycles/pair):",
          ", ".join(f"{n} {ph[k][q] / max(int(st['inner'][k]), 1):.0f} ({100 * ph[k][q] / max(tot, 1):.0f}%)"
                    for q, n in enumerate(names)))

"""Device timeline of the headline fit's working-set rounds without a profiler attached
(HFENS_WS_EVENTS=1: an event per group after every enqueued chunk of rounds): per group, the
time from the SMO batch's start to the end of each chunk, the last useful round and the batch end.
With HFENS_TRACE_HOST=1 the host marks of the same fit follow (ms since develop() was entered;
the batch's start event is recorded at the host mark ws_groups_ready)."""
import os
import sys

os.environ["HFENS_WS_EVENTS"] = "1"
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils import timing  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
for rep in range(6):
    timing._MARKS.clear()
    develop(Xd, yd, Xs, ys, names, device=dev, evaluate=False, timer=StageTimer(enabled=False))
    torch.cuda.synchronize()
    marks = list(timing._MARKS)
    ev = smo.LAST_WS_EVENTS
    st = smo.LAST_WS_STATS
    if rep < 3:
        continue
    print(f"fit {rep}: chunk {ev['chunk']} rounds per mark")
    for gi, mk in enumerate(ev["rounds"]):
        t = [ev["start"].elapsed_time(e) for e in mk]
        grp = st["groups"][gi]
        outer = [int(st["outer"][k]) for k in grp]
        print(f"  group {gi} ({len(grp)} problems, rounds max {max(outer)}): "
              + " ".join(f"{x:.2f}" for x in t))
    if marks:
        t0 = marks[0][1]
        print("  host: " + " ".join(f"{k}={1e3 * (v - t0):.1f}" for k, v in marks))

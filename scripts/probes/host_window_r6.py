"""Host cost of the window before the SVC cascade parts are enqueued (round 6): cProfile of
plan_stacking, LassoCV's prelude up to the early speculation, and prelaunch_stack (the SVC batch),
over 3 warm fits of the bench shape."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import stack_trainer  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
torch.set_num_threads(1)
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
prof = {k: cProfile.Profile() for k in ("plan_stacking", "prelaunch_stack", "prelaunch_bases")}
wall = {k: [] for k in prof}
on = [False]


def wrap(mod, name):
    orig = getattr(mod, name)

    def w(*a, **k):
        if not on[0]:
            return orig(*a, **k)
        t = time.perf_counter()
        prof[name].enable()
        try:
            return orig(*a, **k)
        finally:
            prof[name].disable()
            wall[name].append(1e3 * (time.perf_counter() - t))
    setattr(mod, name, w)


wrap(stack_trainer, "plan_stacking")
wrap(stack_trainer, "prelaunch_stack")
wrap(stack_trainer, "prelaunch_bases")
for i in range(8):
    on[0] = i >= 5
    develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)
torch.cuda.synchronize()
for k, p in prof.items():
    print(f"==== {k}: wall ms under cProfile {[round(x, 2) for x in wall[k]]}")
    st = pstats.Stats(p)
    st.sort_stats("tottime").print_stats(25)
# the same three without the profiler
on[0] = False
times = {k: [] for k in prof}
for k in prof:
    orig = getattr(stack_trainer, k)


def timed(name):
    orig = getattr(stack_trainer, name)

    def w(*a, **kw):
        t = time.perf_counter()
        try:
            return orig(*a, **kw)
        finally:
            times[name].append(1e3 * (time.perf_counter() - t))
    setattr(stack_trainer, name, w)


for k in prof:
    timed(k)
for i in range(6):
    develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)
torch.cuda.synchronize()
print("wall ms without the profiler:", {k: [round(x, 3) for x in v[2:]] for k, v in times.items()})

"""cProfile of the host work between the LassoCV path launch and the SVC batch's first rounds:
stack_trainer.prelaunch_stack (the stacking fit enqueued on the speculative selection), 3 fits."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import stack_trainer  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
orig = stack_trainer.prelaunch_stack
pr = cProfile.Profile()
on = [False]


def wrapped(*a, **k):
    if not on[0]:
        return orig(*a, **k)
    pr.enable()
    try:
        return orig(*a, **k)
    finally:
        pr.disable()


stack_trainer.prelaunch_stack = wrapped
for i in range(7):
    on[0] = i >= 4
    develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(45)

"""cProfile of the headline fit's host window between the LassoCV read-back and the first
working-set round (host marks lasso_fit → ws_groups_ready): the host-bound setup of the SMO."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils import timing  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
pr = cProfile.Profile()
state = {"on": False, "armed": False}
orig = timing.hmark


def hmark(name):
    if state["armed"] and name == "lasso_fit" and not state["on"]:
        pr.enable()
        state["on"] = True
    elif state["on"] and name == "ws_groups_ready":
        pr.disable()
        state["on"] = False
        state["armed"] = False


timing.hmark = hmark
for rep in range(4):
    state["armed"] = rep >= 2
    develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)
    torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(25)

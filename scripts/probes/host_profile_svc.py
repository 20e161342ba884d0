"""cProfile of the stacking fit's SVC prelaunch (smo.launch_svc_batch: expansion, gather, cascade
parts, solver groups, rounds enqueued) in the headline step — the host window that the SVC's
device chain waits for."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
pr = cProfile.Profile()
orig = smo.launch_svc_batch
active = [False]


def wrapped(*a, **k):
    if active[0]:
        pr.enable()
    try:
        return orig(*a, **k)
    finally:
        pr.disable()


smo.launch_svc_batch = wrapped
import hfens.models.stack_trainer as stt  # noqa: E402
if hasattr(stt, "launch_svc_batch"):
    stt.launch_svc_batch = wrapped


def step():
    return develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False))


for _ in range(4):
    step()
torch.cuda.synchronize()
active[0] = True
for _ in range(5):
    step()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(45)

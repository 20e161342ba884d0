"""Host work of the headline fit from develop() entry until the SVC cascade parts are enqueued
(the device's critical chain waits on it: r6 timeline, parts enqueued ≈ 3.4 ms into the fit).
cProfile over that window only (enabled at develop() entry, disabled when smo._cascade_seed
returns), 3 warm fits of the bench shape; prints the top functions by own and cumulative time,
and the window's wall time without the profiler.  Usage: python scripts/probes/preparts_profile.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens import pipeline  # noqa: E402
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import smo  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
torch.set_num_threads(1)
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
prof = cProfile.Profile()
state = dict(on=False, t0=0.0, walls=[], profile=False)
_orig_seed = smo._cascade_seed


def seed_wrap(*a, **k):
    out = _orig_seed(*a, **k)
    if state["on"]:
        if state["profile"]:
            prof.disable()
        state["walls"].append(1e3 * (time.perf_counter() - state["t0"]))
        state["on"] = False
    return out


smo._cascade_seed = seed_wrap
_orig_develop = pipeline.develop


def run(profile):
    state.update(on=True, profile=profile, t0=time.perf_counter())
    if profile:
        prof.enable()
    _orig_develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)
    if state["on"] and profile:   # (no cascade this fit)
        prof.disable()
    state["on"] = False


for i in range(5):
    run(False)
torch.cuda.synchronize()
state["walls"].clear()
for i in range(8):
    run(False)
    torch.cuda.synchronize()
print("window wall ms without the profiler:", [round(w, 2) for w in state["walls"]])
state["walls"].clear()
for i in range(3):
    run(True)
    torch.cuda.synchronize()
print("window wall ms under cProfile:", [round(w, 2) for w in state["walls"]])
st = pstats.Stats(prof)
rows = [(tt / 3 * 1e6, ct / 3 * 1e6, nc / 3, f"{os.path.basename(k[0])}:{k[1]}({k[2]})")
        for k, (cc, nc, tt, ct, _) in st.stats.items()]
print("\nper fit: own µs, cumulative µs, calls, function — by own time")
for r in sorted(rows, key=lambda r: -r[0])[:45]:
    print(f"{r[0]:8.1f} {r[1]:8.1f} {r[2]:6.0f}  {r[3]}")
print("\nby cumulative time")
for r in sorted(rows, key=lambda r: -r[1])[:70]:
    print(f"{r[0]:8.1f} {r[1]:8.1f} {r[2]:6.0f}  {r[3]}")
print("\ncallers of the most-called tensor methods (per fit: calls, own µs of the callee under that caller)")
for k, (cc, nc, tt, ct, callers) in st.stats.items():
    if k[2] in ("<method 'to' of 'torch._C.TensorBase' objects>", "<method 'index_select' of 'torch._C.TensorBase' objects>",
                "<method 'pin_memory' of 'torch._C.TensorBase' objects>", "<method 'sum' of 'torch._C.TensorBase' objects>",
                "<built-in method torch.empty>", "<built-in method torch.zeros>", "<built-in method torch.where>"):
        print(k[2])
        for ck, cv in sorted(callers.items(), key=lambda t: -t[1][2]):
            print(f"    {cv[1] / 3:5.1f} {cv[2] / 3 * 1e6:7.1f}  {os.path.basename(ck[0])}:{ck[1]}({ck[2]})")

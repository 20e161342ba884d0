"""Per-step record of the headline fit (the ≈ 13 ms step outliers): N timed develop()
steps of the bench shape, each with its wall time and the mechanisms that could cost a step —
speculation miss, cooperative-LR / SMO fallbacks, working-set re-solve, GBDT persist fallback,
allocator growth (reserved bytes), Python GC collections, host CPU time, and the process's
involuntary context switches (a descheduled host thread stalls every launch behind it).
Usage: python scripts/probes/step_outliers.py [steps] > log"""
import gc
import json
import os
import resource
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.models import hist_gbdt, logreg_solver, smo, stack_trainer  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
# SYNC=0: steps back to back as bench.py times them (a step is host return to host return)
SYNC = os.environ.get("SYNC", "1") != "0"
dev = torch.device("cuda")
torch.set_num_threads(int(os.environ.get("HFENS_HOST_THREADS", "1")))
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
gcn = [0]
gcinfo = {"gen": -1, "ms": 0.0, "t": 0.0}


def _gc_cb(phase, info):
    if phase == "start":
        gcn[0] += 1
        gcinfo["gen"] = max(gcinfo["gen"], info["generation"])
        gcinfo["t"] = time.perf_counter()
    else:
        gcinfo["ms"] += 1e3 * (time.perf_counter() - gcinfo["t"])


gc.callbacks.append(_gc_cb)
if os.environ.get("GC_OFF", "0") == "1":
    gc.disable()


def fit():
    return develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)


for _ in range(5):
    fit()
torch.cuda.synchronize()
if os.environ.get("HFENS_GC_FREEZE", "1") != "0":
    gc.collect()
    gc.freeze()
recs = []
for k in range(steps):
    for d in (smo.LAST_SMO_INFO, logreg_solver.LAST_PATH, hist_gbdt.LAST_PATH, stack_trainer.LAST_PRELAUNCH):
        for key in ("ws_resolve", "coop_fallback", "persist_fallback", "spec_miss"):
            d.pop(key, None)
    g0, r0, a0 = gcn[0], torch.cuda.memory_reserved(dev), torch.cuda.memory_allocated(dev)
    gcinfo.update(gen=-1, ms=0.0)
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    if SYNC:
        torch.cuda.synchronize()
    t0 = time.perf_counter() if SYNC or k == 0 else t_prev
    c0 = time.process_time()
    fit()
    if SYNC:
        torch.cuda.synchronize()
    t_prev = time.perf_counter()
    dt = 1e3 * (t_prev - t0)
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    recs.append(dict(step=k, ms=round(dt, 3), cpu_ms=round(1e3 * (time.process_time() - c0), 2),
                     nivcsw=ru1.ru_nivcsw - ru0.ru_nivcsw, nvcsw=ru1.ru_nvcsw - ru0.ru_nvcsw,
                     gc=gcn[0] - g0, gc_gen=gcinfo["gen"], gc_ms=round(gcinfo["ms"], 3),
                     reserved_growth=torch.cuda.memory_reserved(dev) - r0,
                     allocated_growth=torch.cuda.memory_allocated(dev) - a0,
                     spec_miss=stack_trainer.LAST_PRELAUNCH.get("spec_miss", 0),
                     ws_resolve=bool(smo.LAST_SMO_INFO.get("ws_resolve")),
                     coop_fallback=bool(smo.LAST_SMO_INFO.get("coop_fallback")) or bool(logreg_solver.LAST_PATH.get("coop_fallback")),
                     persist_fallback=hist_gbdt.LAST_PATH.get("persist_fallback", 0)))
    print(json.dumps(recs[-1]), flush=True)
ms = sorted(r["ms"] for r in recs)
med = ms[len(ms) // 2]
print(json.dumps(dict(summary=True, steps=steps, min=ms[0], median=med, max=ms[-1], ratio=round(ms[-1] / med, 3),
                      reserved_total_growth=sum(r["reserved_growth"] for r in recs),
                      allocated_total_growth=sum(r["allocated_growth"] for r in recs),
                      over_1_25=[r for r in recs if r["ms"] > 1.25 * med])), flush=True)

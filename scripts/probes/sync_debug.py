"""Which host lines synchronise with the device during one headline step?  torch's sync debug mode
warns on every synchronising tensor operation; each warning is printed with the framework frames
of its stack.  (Implicit synchronisation inside the runtime, e.g. an allocation, is not seen.)"""
import os
import sys
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))


def step():
    return develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)


for _ in range(3):
    step()
torch.cuda.synchronize()
seen = []


def show(message, category, filename, lineno, file=None, line=None):
    fr = [f for f in traceback.extract_stack()[:-1] if "/hfens/" in f.filename or "machine-learning" in f.filename]
    seen.append((str(message)[:80], [f"{os.path.basename(f.filename)}:{f.lineno} {f.name}" for f in fr[-4:]]))


warnings.showwarning = show
warnings.simplefilter("always")
torch.cuda.set_sync_debug_mode("warn")
step()
torch.cuda.set_sync_debug_mode(0)
torch.cuda.synchronize()
for m, fr in seen:
    print(m, "|", " <- ".join(reversed(fr)))
print("synchronising ops:", len(seen))

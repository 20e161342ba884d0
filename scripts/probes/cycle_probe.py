"""Which reference cycles hold device memory after a headline fit (round 6: ~77 MB per fit stayed
allocated until a full GC, profiles/r6_runs/r6o)?  One warm fit under gc.DEBUG_SAVEALL: every
object the collector finds unreachable is kept in gc.garbage; print the CUDA bytes and the
containers (dict keys, closure names) of those cycles."""
import collections
import gc
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort  # noqa: E402
from hfens.pipeline import develop  # noqa: E402
from hfens.utils.timing import StageTimer  # noqa: E402

dev = torch.device("cuda")
Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
Xd, yd, Xs, ys = (torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys))
for _ in range(3):
    develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)
torch.cuda.synchronize()
gc.collect()
a0 = torch.cuda.memory_allocated(dev)
gc.disable()
develop(Xd, yd, Xs, ys, names, device=dev, timer=StageTimer(enabled=False), evaluate=False)
torch.cuda.synchronize()
a1 = torch.cuda.memory_allocated(dev)
gc.set_debug(gc.DEBUG_SAVEALL)
n = gc.collect()
a2 = torch.cuda.memory_allocated(dev)
print(f"allocated after fit +{(a1 - a0) / 1e6:.1f} MB; unreachable objects {n}; gc.garbage {len(gc.garbage)}")
cuda = [o for o in gc.garbage if isinstance(o, torch.Tensor) and o.is_cuda]
print(f"CUDA tensors in cycles: {len(cuda)}, {sum(t.untyped_storage().nbytes() for t in cuda) / 1e6:.1f} MB (storage)")
types_ = collections.Counter(type(o).__name__ for o in gc.garbage)
print("types:", types_.most_common(15))
keyc = collections.Counter()
for o in gc.garbage:
    if isinstance(o, dict):
        keyc[tuple(sorted(map(str, o.keys()))[:8])] += 1
print("dict key sets (first 8 keys):")
for k, v in keyc.most_common(25):
    print(f"  {v} × {k}")
fn = collections.Counter(o.__qualname__ + " @ " + os.path.basename(o.__code__.co_filename) for o in gc.garbage
                         if isinstance(o, types.FunctionType))
print("closures:")
for k, v in fn.most_common(40):
    print(f"  {v} × {k}")
gc.set_debug(0)
gc.garbage.clear()
gc.collect()
print(f"allocated after clearing: {(torch.cuda.memory_allocated(dev) - a0) / 1e6:.1f} MB over the pre-fit level")

"""Time the Nyström map's RBF matrix at config-3 scale: native rbf_f64 (ops/csrc/nystrom.hip) vs
the library GEMM form, and the whole map (K·T).  Usage: python scripts/probes/rbf_probe.py [l] [m]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from hfens.models import svc_lowrank  # noqa: E402

l = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 512
Z = torch.randn(l, 17, dtype=torch.float64, device="cuda")
idx = torch.randperm(l, device="cuda")[:m]
L = Z[idx]


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


res = {}
for native in (True, False):
    svc_lowrank.NATIVE_RBF = native
    res[native] = (t(lambda: svc_lowrank._rbf(Z, L, 1 / 17)), t(lambda: svc_lowrank.nystrom_map(Z, idx, 1 / 17), 3))
svc_lowrank.NATIVE_RBF = True
gb = l * m * 8 / 1e9
print(f"rbf {l}x{m}: native {res[True][0]:.2f} ms ({gb / res[True][0]:.2f} TB/s of K written), "
      f"library {res[False][0]:.2f} ms; whole map: native {res[True][1]:.2f} ms, library {res[False][1]:.2f} ms")

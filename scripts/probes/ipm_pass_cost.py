"""Per-pass cost of the interior point's row passes at config-3 shape (l = 1M, r = 428), alone on
the GPU: Φ·W (phi_gemv_f32), Φᵀ·V (phit_f32), the weighted Gram (library block-upper f64 path and
the native f64 kernel), with the bytes each moves and the achieved rate."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.models import svc_lowrank as sl  # noqa: E402

dev = torch.device("cuda")
l, r = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000, 428
P32 = torch.randn(l, r, device=dev)
Phi = P32.to(torch.float64)
d = torch.rand(l, dtype=torch.float64, device=dev) + 0.1


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


for k in (1, 2):
    W = torch.randn(r, k, dtype=torch.float64, device=dev)
    V = torch.randn(l, k, dtype=torch.float64, device=dev)
    ms = t(lambda: sl._phi_mv(Phi, W, P32))
    print(f"phi_gemv_f32 k={k}: {ms:.3f} ms  {(l * r * 4 + l * k * 8) / ms / 1e9:.2f} TB/s", flush=True)
    ms = t(lambda: sl._phit(Phi, V, P32))
    print(f"phit_f32 k={k}: {ms:.3f} ms  {(l * r * 4 + l * k * 8) / ms / 1e9:.2f} TB/s", flush=True)
sl.GRAM = "f64"
for bs in (128, 96, 64, 32):
    sl.SYRK_BLOCK = bs
    ms = t(lambda: sl._weighted_gram(Phi, d, P32), 5)
    print(f"weighted gram (library block-upper f64, block {bs}): {ms:.3f} ms", flush=True)
sl.SYRK_BLOCK = 128
S0 = sl._weighted_gram(Phi, d, P32)
sc = sl._scaled_rows(Phi, d, P32)
ms = t(lambda: sl._scaled_rows(Phi, d, P32), 5)
print(f"scaled rows: {ms:.3f} ms", flush=True)
sl.NATIVE_SYRK = True
ms = t(lambda: sl._weighted_gram(Phi, d, P32), 5)
print(f"weighted gram (native f64 wsyrk): {ms:.3f} ms  {l * r * r * 1.0 / ms / 1e9:.1f} TFLOP/s (upper)", flush=True)
sl.NATIVE_SYRK = False
sl.GRAM = "f64x"
ms = t(lambda: sl._weighted_gram(Phi, d, P32), 5)
S1 = sl._weighted_gram(Phi, d, P32)
err = float(((S1 - S0).abs().max() / S0.abs().max()))
print(f"weighted gram (native f64 from f32 Φ): {ms:.3f} ms  max rel diff vs library {err:.2e}", flush=True)

"""Donor-search throughput: the packed-FMA filter kernel vs the bf16 matrix-core filter
(knn.hip knn_donor_fast_kernel / knn_donor_mfma_kernel) on Table S1-shaped rows, receivers = rows
with a missing cell, donors = every row; pairs/s = receivers × donors / kernel time."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens import ops  # noqa: E402
from hfens.io.synth import make_hf_cohort  # noqa: E402

dev = torch.device("cuda")
E = ops.ext()
for n in [int(a) for a in sys.argv[1:]] or [10000, 100000]:
    F = 40
    X, _, _ = make_hf_cohort(n, F, seed=n, nan_frac=0.02)
    mu = np.nanmean(X, 0)
    miss = np.isnan(X)
    Xc = np.where(miss, 0.0, X - mu).astype(np.float32)
    bits = (miss.astype(np.uint64) << np.arange(F, dtype=np.uint64)).sum(1).astype(np.uint64).view(np.int64)
    rows = np.nonzero(miss.any(1))[0]
    slot = np.full((rows.shape[0], 8), -1, dtype=np.int32)
    for i, r in enumerate(rows):
        c = np.nonzero(miss[r])[0][:8]
        slot[i, :c.shape[0]] = c
    s = ops.stream_ptr(dev)
    R = torch.as_tensor(Xc[rows], device=dev).contiguous()
    rm = torch.as_tensor(bits[rows], device=dev)
    D = torch.as_tensor(Xc, device=dev).contiguous()
    dm = torch.as_tensor(bits, device=dev)
    sl = torch.as_tensor(slot, device=dev)
    nr, nd = R.shape[0], D.shape[0]
    best = torch.empty(nr, 8, dtype=torch.int64, device=dev)
    alt = torch.empty(nr, 8, dtype=torch.int32, device=dev)
    wd = np.zeros(1, dtype=np.int64)
    E.knn_mfma_item_words(F, wd.ctypes.data)
    items = torch.empty(nd * int(wd[0]), dtype=torch.int32, device=dev)
    ny = torch.empty(nd, dtype=torch.float32, device=dev)
    res = {}
    for kind in ("fast", "mfma", "fast", "mfma"):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        if kind == "fast":
            E.knn_donors(R.data_ptr(), rm.data_ptr(), nr, D.data_ptr(), dm.data_ptr(), nd, F, sl.data_ptr(),
                         best.data_ptr(), alt.data_ptr(), 0, 0, s)
        else:
            E.knn_mfma_prep(D.data_ptr(), dm.data_ptr(), nd, F, items.data_ptr(), ny.data_ptr(), s)
            E.knn_donors_mfma(R.data_ptr(), rm.data_ptr(), nr, D.data_ptr(), dm.data_ptr(), nd, F, sl.data_ptr(),
                              best.data_ptr(), alt.data_ptr(), 0, 0, items.data_ptr(), ny.data_ptr(), s)
        e1.record()
        torch.cuda.synchronize()
        res[kind] = e0.elapsed_time(e1)
    for kind, ms in res.items():
        print(f"n={n} receivers={nr} {kind}: {ms:.3f} ms  {nr * nd / ms / 1e6:.1f} G pairs/s", flush=True)

"""BASELINE config 1: single-patient predict_proba latency on the shipped checkpoint (excludes
unpickle, like the 85 µs numpy baseline).  Prints p50/p99 in µs for the native host predictor
(ops/csrc/host.hip stack_predict_host) and the generic per-model torch path."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
torch.set_num_threads(1)
from hfens.cli.predict_hf import PATIENT_PARAMS  # noqa: E402
from hfens.io.checkpoint import load_checkpoint  # noqa: E402


def lat(fn, reps=3000):
    for _ in range(100):
        fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return round(np.percentile(ts, 50) * 1e6, 1), round(np.percentile(ts, 99) * 1e6, 1)


def main():
    dev = sys.argv[1] if len(sys.argv) > 1 else "cpu"
    clf = load_checkpoint(device=dev)
    x = torch.tensor([[float(v) for v in PATIENT_PARAMS.values()]], dtype=torch.float64, device=dev)
    out = {"device": dev, "p": float(clf.predict_proba(x)[0, 1])}
    sync = torch.cuda.synchronize if dev != "cpu" else (lambda: None)
    out["native_p50_p99_us"] = lat(lambda: (clf.predict_proba(x), sync()))
    clf.HOST_NATIVE_MAX_ROWS = -1
    out["generic_p50_p99_us"] = lat(lambda: (clf.predict_proba(x), sync()), reps=500)
    out["generic_p"] = float(clf.predict_proba(x)[0, 1])
    out["baseline_p50_us"] = 85.0
    print(json.dumps(out))


if __name__ == "__main__":
    main()

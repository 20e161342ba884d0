"""Phase split of one GBDT boosting stage (gbdt_stump_stage, 1M x 40, 1 and 5 models): the
in-kernel s_memtime stamps of stage HFENS_GBDT_STAGE_PROF (split done / first sub-tile applied /
histogram done / published, cycles since the workgroup started the stage), per workgroup, plus the
stage loop's event time without stamps."""
import os
import sys

os.environ.setdefault("HFENS_GBDT_STAGE_PROF", "50")
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hfens.io.synth import make_hf_cohort_device  # noqa: E402
from hfens.models import hist_gbdt  # noqa: E402
from hfens.models.gbdt import GradientBoostingClassifier  # noqa: E402
from hfens.models.hist_gbdt import fit_gbdt_batch  # noqa: E402

dev = torch.device("cuda", 0)
T = 100
GHZ = float(os.environ.get("PROBE_GHZ", "2.4"))
rows = int(os.environ.get("PROBE_ROWS", "1000000"))
X, y = make_hf_cohort_device(rows, 40, seed=7, rows=(0, rows), device=dev)
for B in (1, 5):
    for prof in (False, True):
        hist_gbdt.PROFILE_STAGE_T = 50 if prof else -1
        loop = []
        for rep in range(4):
            ms = [GradientBoostingClassifier(n_estimators=T, max_depth=1, random_state=1 + k) for k in range(B)]
            fit_gbdt_batch(ms, X, y)
            torch.cuda.synchronize()
            e0, e1 = hist_gbdt.GRAPH_INFO["loop_events"]
            loop.append(e0.elapsed_time(e1))
        us = 1e3 * sorted(loop)[1] / (T + 2)
        if not prof:
            print(f"rows {rows} B {B}: {us:.1f} us/stage (no stamps), persist={hist_gbdt.GRAPH_INFO.get('persist')}")
            continue
        st = hist_gbdt.LAST_STAGE_PROF["stamps"].astype(np.float64) / (GHZ * 1e3)   # µs
        q = lambda c: np.percentile(st[:, c], [50, 90, 100])  # noqa: E731
        print(f"  stamps (us, p50/p90/max over {st.shape[0]} workgroups): split {q(0).round(1)}  "
              f"hist {q(2).round(1)}  published {q(3).round(1)}  "
              f"[wave 0 summed over sub-tiles: apply {q(1).round(1)}  MFMA part {q(4).round(1)}  wide-atomic part {q(5).round(1)}]")

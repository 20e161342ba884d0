"""Median device / host timeline marks over the traced fits of a HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1
bench run (stderr file), skipping the first SKIP fits.  Usage: python scripts/probes/tl_summary.py
ERRFILE [SKIP]"""
import re
import sys
from statistics import median

path = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev, host = [], []
for line in open(path):
    if line.startswith("[dev]"):
        dev.append(dict((k, float(v)) for k, v in re.findall(r"(\w+)=([0-9.]+)", line)))
    elif line.startswith("[host]"):
        d = {}
        for k, v in re.findall(r"(\w+)=([0-9.]+)", line):
            d.setdefault(k, float(v))      # first occurrence (ws_chunk repeats)
        host.append(d)
dev, host = dev[skip:], host[skip:]
keys = ["lasso_spec", "svc_parts_done", "svc_smo_done", "svc_platt", "svc_oof", "lr_kernel", "gbc_done", "lasso_cv_path", "meta", "stack_fit"]
print(f"fits {len(dev)} dev medians: " + " ".join(f"{k}={median(d[k] for d in dev if k in d):.2f}" for k in keys if any(k in d for d in dev)))
if all("svc_platt_dec" in d and "svc_smo_done" in d for d in dev):
    print(f"tail medians: dec {median(d['svc_platt_dec'] - d['svc_smo_done'] for d in dev):.3f} "
          f"platt {median(d['svc_platt'] - d['svc_platt_in'] for d in dev):.3f} "
          f"smo→stack_fit {median(d['stack_fit'] - d['svc_smo_done'] for d in dev):.3f}")
if all(k in d for d in dev for k in ("svc_oof", "lr_launch", "lr_kernel", "meta", "stack_fit")):
    print(f"meta medians: oof→lr_kernel {median(d['lr_kernel'] - d['svc_oof'] for d in dev):.3f} "
          f"lr_launch→lr_kernel {median(d['lr_kernel'] - d['lr_launch'] for d in dev):.3f} "
          f"lr_kernel→meta {median(d['meta'] - d['lr_kernel'] for d in dev):.3f} "
          f"meta→stack_fit {median(d['stack_fit'] - d['meta'] for d in dev):.3f}")
hk = ["develop", "lasso_spec_launched", "svc_cascade_seeded", "ws_groups_ready", "svc_solve_enqueued", "lasso_best_read", "svc_host_read"]
print("host medians (ms after develop): " + " ".join(
    f"{k}={median(h[k] - h['develop'] for h in host if k in h and 'develop' in h):.2f}" for k in hk[1:] if any(k in h for h in host)))

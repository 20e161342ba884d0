"""Host-side tail of the traced stacking fits (HFENS_TRACE_HOST=1 stderr): median ms of each mark
after svc_early_wait, and of the [host-meta] marks after meta_in.  Usage: tail_host.py ERRFILE [SKIP]"""
import re
import sys
from statistics import median

path = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
fits, meta = [], []
for line in open(path):
    if line.startswith("[host]"):
        d = {}
        for k, v in re.findall(r"(\w+)=([0-9.]+)", line):
            d.setdefault(k, float(v))
        fits.append(d)
    elif line.startswith("[host-meta]"):
        meta.append(dict((k, float(v)) for k, v in re.findall(r"(\w+)=([0-9.]+)", line)))
fits, meta = fits[skip:], meta[skip:]
ks = ["svc_early_wait", "svc_early_synced", "svc_host_read", "svc_platt_read", "svc_set_fitted", "svc_finished",
      "bases_resolved", "bases_resolved_early"]
print("host tail after svc_early_wait: " + " ".join(
    f"{k}={median(d[k] - d['svc_early_wait'] for d in fits if k in d and 'svc_early_wait' in d):.3f}" for k in ks[1:]
    if any(k in d and 'svc_early_wait' in d for d in fits)))
if meta:
    print("host-meta: " + " ".join(f"{k}={median(m[k] for m in meta if k in m):.3f}" for k in meta[0]))

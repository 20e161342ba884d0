"""Sweep the fused stack kernel's workgroup shape on the shipped checkpoint (GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rows = sys.argv[1] if len(sys.argv) > 1 else "100000000"
for w in ("8", "12", "16"):
    env = dict(os.environ, HFENS_STACK_WAVES=w)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "infer", "--rows", rows,
                        "--steps", "5", "--warmup", "1"], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not line:
        print(w, "FAILED", r.stderr[-2000:])
        sys.exit(1)
    d = json.loads(line[-1])
    print(json.dumps({"waves": w, "rows_per_s": d["value"], "ms": d["ms_per_step"],
                      "stream_rows_per_s": d["host_stream_rows_per_sec"], "err": d["max_abs_err_vs_per_model_path"]}))

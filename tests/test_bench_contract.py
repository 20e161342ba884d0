"""bench.py's driver contract on the CPU: ONE JSON line from rank 0 with the required keys, for one
process and for a 2-rank torchrun over gloo (rendezvous on 127.0.0.1)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config")
CONFIG_KEYS = ("model", "global_batch", "seq_len", "parallelism")


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{") and '"metric"' in l]


def _check(d, n):
    for k in KEYS:
        assert k in d, k
    for k in CONFIG_KEYS:
        assert k in d["config"], k
    assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}"
    assert d["metric"] == "train_rows_per_sec" and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["steps"] == 1 and d["warmup"] == 0
    assert abs(d["value"] - d["config"]["global_batch"] * 1000.0 / d["ms_per_step"]) < 1e-3 * d["value"] + 1e-6


def _env():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_bench_single_process_json_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--rows", "600"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check(lines[0], 1)


def test_bench_torchrun_two_ranks_one_json_line():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "1",
           "--warmup", "0", "--rows", "600"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    _check(lines[0], 2)

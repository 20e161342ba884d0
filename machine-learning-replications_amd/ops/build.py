"""In-tree build of the gfx950 HIP extension ``hfens/ops/_hfens_hip*.so``.

Every ``csrc/*.hip`` translation unit is compiled by ``hipcc --offload-arch=gfx950``
(CDNA4 only; no CUDA shims, no hipify) and linked with the pybind11 bindings
against the HIP runtime that PyTorch-ROCm itself loads (``torch/lib/libamdhip64.so``,
same soname as /opt/rocm's) so there is exactly one HIP runtime in the process.
Object files are cached by content hash under ``ops/_build`` (git-ignored); the
resulting ``.so`` lives next to this file so it travels with the repo snapshot.

Usage: ``python -m hfens.ops.build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# fast contraction everywhere except where a kernel says `#pragma clang fp contract(off)` (the
# libsvm-arithmetic SMO kernels, the interior point's bit-identical tails): plain `fast` ignores
# the pragma
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            "-Wno-unused-result", "-ffp-contract=fast-honor-pragmas"]


def _torch_lib() -> str:
    import importlib.util
    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _pybind_inc() -> str:
    import pybind11
    return pybind11.get_include()


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(HERE, "_hfens_hip" + suffix)


def _sources():
    hips = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    return [os.path.join(CSRC, f) for f in hips] + [os.path.join(CSRC, "bindings.cpp")]


def _headers_digest() -> str:
    h = hashlib.sha1()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".h", ".inc")):
            h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()


def _compile(src: str, hdr: str) -> str:
    data = open(src, "rb").read()
    key = hashlib.sha1(data + hdr.encode() + " ".join(CXXFLAGS).encode()).hexdigest()[:16]
    obj = os.path.join(BUILD, os.path.basename(src) + f".{key}.o")
    if os.path.exists(obj):
        return obj
    inc = ["-I", CSRC, "-I", _pybind_inc(), "-I", sysconfig.get_paths()["include"]]
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC] + CXXFLAGS + inc + lang + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hdr = _headers_digest()
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr), srcs))
    out = ext_path()
    stamp = hashlib.sha1("".join(objs).encode()).hexdigest()
    stamp_file = os.path.join(BUILD, "link.stamp")
    if not force and os.path.exists(out) and os.path.exists(stamp_file) and open(stamp_file).read() == stamp:
        return out
    tl = _torch_lib()
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs + [
        "-L", tl, "-lamdhip64", f"-Wl,-rpath,{tl}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    with open(stamp_file, "w") as f:
        f.write(stamp)
    if verbose:
        print(f"[hfens.ops.build] {out}")
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    build(force=a.force, jobs=a.j)

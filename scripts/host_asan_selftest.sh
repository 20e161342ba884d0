#!/bin/bash
# Build the host helpers + self-test with ASan/UBSan (host code only: each -fsanitize= follows
# -Xarch_host, so no device code is instrumented) and run it on the CPU.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${TMPDIR:-/tmp}/hfens_host_selftest"
CSRC="$ROOT/machine-learning-replications_amd/ops/csrc"
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O1 -g -fno-omit-frame-pointer \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  "$CSRC/host.hip" -x c++ "$ROOT/machine-learning-replications_amd/ops/selftest/host_selftest.cpp" -o "$OUT"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1 "$OUT"

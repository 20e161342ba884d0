#!/bin/bash
# round 4: config 3 (1M rows, full ensemble) with this round's kernels (f64-exact KNN, multi-workgroup
# Cholesky, exact SVC up to 150k points per problem)
set -o pipefail
D=gpurun_out/r4m
mkdir -p $D
timeout -k 10 600 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $D/cfg3.json 2> $D/cfg3.err || { echo "cfg3 failed"; tail -30 $D/cfg3.err; exit 1; }
cat $D/cfg3.json

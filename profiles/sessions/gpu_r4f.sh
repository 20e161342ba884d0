#!/bin/bash
# round 4: headline host marks + kernel timeline of one fit (q = 1024 default)
set -o pipefail
D=gpurun_out/r4f
mkdir -p $D
HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 10 --warmup 5 > $D/bench_marks.json 2> $D/bench_marks.err || { echo "bench failed"; tail -30 $D/bench_marks.err; exit 1; }
grep "\[host\]" $D/bench_marks.err | tail -3
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/trace -o tb --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
f=$(find $D/trace -name "*kernel_trace.csv" | head -1)
python scripts/probes/timeline.py $f > $D/timeline.txt 2>&1 || { tail -20 $D/timeline.txt; exit 1; }
head -60 $D/timeline.txt

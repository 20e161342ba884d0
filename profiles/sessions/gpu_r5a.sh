#!/bin/bash
# Round 5, first GPU session: the driver's headline command with the round-4 synchronous base fits
# (HFENS_DEVICE_BASES=0 HFENS_BIN_AHEAD=0) and with the host-sync-free ones, device/host timelines
# of both, the full GPU suite, and PMC counters for the working-set SMO kernel (one pass per group).
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
B0="HFENS_DEVICE_BASES=0 HFENS_BIN_AHEAD=0"
env $B0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_r4path.json 2> $O/bench_r4path.err || { echo "bench r4 path failed"; tail -20 $O/bench_r4path.err; exit 1; }
cut -c1-300 $O/bench_r4path.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
env $B0 HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --steps 6 --warmup 3 > $O/timeline_r4path.json 2> $O/timeline_r4path.err || { echo "timeline r4 failed"; tail -20 $O/timeline_r4path.err; exit 1; }
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --steps 6 --warmup 3 > $O/timeline.json 2> $O/timeline.err || { echo "timeline failed"; tail -20 $O/timeline.err; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
pass() {  # pass TAG COUNTERS...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/$tag -o p --output-format csv -- python3 bench.py --steps 1 --warmup 1 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  f=$(find $O/$tag -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summary.py $f $O/pmc_$tag.csv "" && rm -rf $O/$tag && head -12 $O/pmc_$tag.csv | cut -c1-300
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD
pass sq3 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE

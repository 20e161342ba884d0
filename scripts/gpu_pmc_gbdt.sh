#!/bin/bash
# PMC counters for the GBDT stage kernel (1M x 40, 100 stumps): one pass per counter group.
set -o pipefail
D=${PMC_DIR:-gpurun_out/pmc_gbdt}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
pass() {  # pass TAG COUNTERS...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $D/$tag -o p --output-format csv -- python3 bench.py ${BENCH_ARGS:---config gbdt --steps 1 --warmup 0} > $D/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $D/$tag.log; exit 1; }
  f=$(find $D/$tag -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summary.py $f $D/$tag.csv "${PMC_MATCH:-}" && rm -rf $D/$tag && cat $D/$tag.csv | cut -c1-400
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD
pass tcc FETCH_SIZE GRBM_GUI_ACTIVE
pass mf SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH

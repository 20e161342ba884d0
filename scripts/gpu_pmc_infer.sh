#!/bin/bash
# PMC counters for the fused inference kernel (counters only: no trace domains in this run).
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --kernel-include-regex stack_infer -d gpurun_out/pmc/a -o a --output-format csv -- python bench.py --config infer --rows 20000000 --steps 1 --warmup 1 > gpurun_out/pmc/a.log 2>&1 || { echo "pmc a failed"; tail -20 gpurun_out/pmc/a.log; }
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex stack_infer -d gpurun_out/pmc/b -o b --output-format csv -- python bench.py --config infer --rows 20000000 --steps 1 --warmup 1 > gpurun_out/pmc/b.log 2>&1 || { echo "pmc b failed"; tail -20 gpurun_out/pmc/b.log; }
ls -R gpurun_out/pmc | head -30

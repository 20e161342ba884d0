#!/bin/bash
# Round 5: counters of the matrix-core KNN filter after the bound rework (n = 100k probe).
set -o pipefail
O=gpurun_out/r5ak
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p1 -o run -- python3 scripts/probes/knn_mfma_probe.py 100000 > $O/p1.log 2>&1 || { echo "p1 failed"; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $O/p2 -o run -- python3 scripts/probes/knn_mfma_probe.py 100000 > $O/p2.log 2>&1 || { echo "p2 failed"; tail -20 $O/p2.log; exit 1; }
for p in p1 p2; do f=$(find $O/$p -name '*counter_collection.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name']
    if 'knn_donor_mfma' not in k: continue
    agg[r['Counter_Name']] += float(r['Counter_Value'])
tiles = 2 * 55369 * 100000 / 1024
for c, v in sorted(agg.items()): print(f"{c:24s} {v:.4g}  per tile-wave {v / tiles:.1f}")
PY
done

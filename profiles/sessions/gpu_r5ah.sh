#!/bin/bash
# Round 5: counters of the matrix-core KNN filter vs the packed-FMA filter (n = 100k probe).
set -o pipefail
O=gpurun_out/r5ah
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/p1 -o run -- python3 scripts/probes/knn_mfma_probe.py 100000 > $O/p1.log 2>&1 || { echo "p1 failed"; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $O/p2 -o run -- python3 scripts/probes/knn_mfma_probe.py 100000 > $O/p2.log 2>&1 || { echo "p2 failed"; tail -20 $O/p2.log; exit 1; }
for p in p1 p2; do f=$(find $O/$p -name '*counter_collection.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name']
    if 'knn_donor' not in k: continue
    agg[(k.split('(')[0][-30:], r['Counter_Name'])] += float(r['Counter_Value'])
for (k, c), v in sorted(agg.items()): print(f"{k:32s} {c:24s} {v:.4g}")
PY
done

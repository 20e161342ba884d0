#!/bin/bash
# Round 6: which threads burn the host CPU during the headline (bench diag busiest_threads, labelled
# with Python thread names; "(native)" = a thread not started by Python), bench x1.
set -o pipefail
O=gpurun_out/r6br
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_1.json 2> $O/b_1.err || { echo "bench failed"; tail -20 $O/b_1.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b_1.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['diag']['host_cpu_fraction'], d['diag']['busiest_threads_cpu_s'])"
HFENS_THREAD_SAMPLE=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_s.json 2> $O/b_s.err || { echo "bench failed"; tail -20 $O/b_s.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b_s.json').read().strip().splitlines()[-1]);print('bench sampled', d['ms_per_step'], d['diag']['busiest_threads_cpu_s'])"
grep "thread-sample" $O/b_s.err

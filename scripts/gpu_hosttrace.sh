#!/bin/bash
set -o pipefail
HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 2>&1 | grep "\[host\]"

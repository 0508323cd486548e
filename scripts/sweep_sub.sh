#!/bin/bash
# c2 bench at several sub-batch sizes (staging footprint vs MALL residency).
set -o pipefail
OUT=gpurun_out/${1:-sweep}; shift
mkdir -p $OUT
for sb in "$@"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --sub-batch $sb > $OUT/bench_$sb.log 2>&1 || { tail $OUT/bench_$sb.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_$sb.log').read().strip().splitlines()[-1]); print($sb, d['value']/1e9, d['roofline']['per_kernel_ms_per_step'])"
done

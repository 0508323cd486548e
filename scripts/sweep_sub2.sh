#!/bin/bash
# c2 bench at several sub-batch sizes (MALL residency of the staging vs per-launch fixed costs).
set -o pipefail
OUT=gpurun_out/${1:-sweep2}; mkdir -p $OUT
for sb in 16777216 8388608 4194304 12582912; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 10 --sub-batch $sb > $OUT/b_$sb.log 2>&1 || { tail $OUT/b_$sb.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/b_$sb.log').read().strip().splitlines()[-1]); print($sb, round(d['value']/1e9,2), d['ms_per_step'], {k: v for k, v in d['roofline']['per_kernel_ms_per_step'].items() if v})"
done
echo all-ok

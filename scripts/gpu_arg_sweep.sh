#!/bin/bash
# c2 bench under several argument sets (parity on).  Usage: bash scripts/gpu_arg_sweep.sh TAG "args" "args" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for A in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 10 $A > $OUT/bench_$i.log 2>&1 || { echo "run $i ($A) failed"; tail -3 $OUT/bench_$i.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$i.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$A', round(d['value']/1e9,2), d['ms_per_step'], (d.get('parity') or {}).get('mismatches'), {k: v for k, v in (r.get('per_kernel_ms_per_step') or {}).items() if v})"
done
echo all-ok

#!/bin/bash
# c3 A/B on one box: the in-tree engine vs copycat_amd/diag/$1 (CC_ENGINE_SO).  Usage: bash scripts/gpu_ab_c3.sh LIB TAG
set -o pipefail
OUT=gpurun_out/${2:-ab_c3}; mkdir -p $OUT
A="--workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-e2e"
for run in a b a2 b2; do
  case $run in a|a2) E="";; b|b2) E="CC_ENGINE_SO=copycat_amd/diag/$1";; esac
  env $E timeout -k 10 300 python bench.py $A > $OUT/$run.log 2>&1 || { tail $OUT/$run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$run.log').read().strip().splitlines()[-1]); print('$run', round(d['value']/1e9,3), d['ms_per_step'], {k: v for k, v in d['roofline']['per_kernel_ms_per_step'].items() if v})"
done

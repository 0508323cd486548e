#!/bin/bash
# A/B of an environment knob on one workload, same library: bash scripts/gpu_ab_env2.sh WORKLOAD "ENV=1" TAG [bench args]
set -o pipefail
WL=$1; ENVB=$2; OUT=gpurun_out/${3:-ab_env}; shift 3
mkdir -p $OUT
A="--workload $WL --no-cpu-baseline --no-parity --no-e2e $@"
for run in a b a2 b2; do
  case $run in a|a2) E="";; b|b2) E="$ENVB";; esac
  env $E timeout -k 10 300 python bench.py $A > $OUT/$run.log 2>&1 || { tail $OUT/$run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$run.log').read().strip().splitlines()[-1]); print('$run', round(d['value']/1e9,3), d['ms_per_step'], {k: v for k, v in d['roofline']['per_kernel_ms_per_step'].items() if v})"
done

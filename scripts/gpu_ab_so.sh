#!/bin/bash
# A/B of engine builds on one workload: bench lines (no gate) for the product .so and each named variant .so.
# Usage: bash scripts/gpu_ab_so.sh TAG WORKLOAD_ARGS... -- SO1 SO2 ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
ARGS=()
while [ "$1" != "--" ]; do ARGS+=("$1"); shift; done; shift
i=0
for so in product "$@" product; do
  i=$((i+1))
  if [ "$so" = product ]; then unset CC_ENGINE_SO; else export CC_ENGINE_SO=$so; fi
  timeout -k 10 300 python bench.py "${ARGS[@]}" --no-parity --no-cpu-baseline --no-e2e > $OUT/ab_$i.log 2>&1 || { echo "run $i ($so) failed"; tail -5 $OUT/ab_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/ab_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$so', round(d['value']/1e9,3), d['ms_per_step'], {k:v for k,v in r.get('per_kernel_ms_per_step',{}).items() if v})"
done
echo all-ok

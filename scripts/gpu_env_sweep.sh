#!/bin/bash
# c2 bench under several environment settings (diagnostics / A/B knobs), parity skipped for the diagnostic ones.
# Usage (via gpurun): bash scripts/gpu_env_sweep.sh TAG "ENV=V ..." "ENV=V ..." ...   ("-" = no extra env, parity on)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  if [ "$E" = "-" ]; then EV=""; PA=""; else EV="$E"; PA="--no-parity"; fi
  timeout -k 10 300 env $EV python bench.py --no-cpu-baseline --no-e2e --steps 10 $PA > $OUT/bench_$i.log 2>&1 || { echo "run $i ($E) failed"; tail -3 $OUT/bench_$i.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$i.log').read().strip().splitlines()[-1]); print('$E', round(d['value']/1e9,2), d['ms_per_step'], (d.get('parity') or {}).get('mismatches'), {k: v for k, v in d['roofline']['per_kernel_ms_per_step'].items() if v})"
done
echo all-ok

#!/bin/bash
# Bench lines only (each with its parity gate).  Usage (via gpurun): bash scripts/gpu_benches.sh TAG [workloads...]
set -o pipefail
TAG=${1:-benches}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for w in "$@"; do
  i=$((i+1))
  case $w in
    c2) A="--steps 20 --warmup 2";;
    c3) A="--workload c3 --steps 2 --warmup 1";;
    c3cv) A="--workload c3 --steps 2 --warmup 1 --cv-rate 0.001";;
    c3w) A="--workload c3 --steps 1 --warmup 1 --cv-rate 0.001 --clear-rate 0.0001";;
    c4) A="--workload c4 --steps 50 --warmup 5";;
    c5) A="--workload c5 --steps 4 --warmup 1";;
  esac
  timeout -k 10 900 python -u bench.py $A > $OUT/bench_${w}_$i.log 2>&1 || { echo "bench $w failed"; tail -5 $OUT/bench_${w}_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_${w}_$i.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$w', round(d['value']/1e9,3), d['ms_per_step'], (d.get('parity') or {}).get('mismatches'), {k:v for k,v in (r.get('per_kernel_ms_per_step') or {}).items() if v})"
done
echo all-ok

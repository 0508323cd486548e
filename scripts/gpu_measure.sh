#!/bin/bash
# Round-end style measurement: every workload's bench line (with parity) + kernel trace/counter profiles per workload.
# Usage (via gpurun): bash scripts/gpu_measure.sh TAG [workloads...]  (default: c2 c4 c5 c3)
set -o pipefail
TAG=${1:-m}; shift
WLS=${@:-c2 c4 c5 c3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for w in $WLS; do
  case $w in
    c2) A="--steps 20 --warmup 2"; P="--steps 3 --warmup 1";;
    c3) A="--workload c3 --steps 2 --warmup 1"; P="--workload c3 --steps 1 --warmup 1";;
    c4) A="--workload c4 --steps 50 --warmup 5"; P="--workload c4 --steps 50 --warmup 5";;
    c5) A="--workload c5 --steps 4 --warmup 1"; P="--workload c5 --steps 2 --warmup 1";;
  esac
  timeout -k 10 600 python -u bench.py $A > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log > $OUT/bench_$w.json
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', round(d['value']/1e9,3), d['ms_per_step'], d.get('parity'), (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('pipeline_frac'))" | cut -c1-400
  bash scripts/gpu_prof.sh $TAG/prof_$w $P > $OUT/prof_$w.log 2>&1 || { echo "prof $w failed"; tail -5 $OUT/prof_$w.log; exit 1; }
done
echo all-ok

#!/bin/bash
# c5 diagnostics: k_apply_coord phase clocks per type (diag build), then the c5 bench (events A/B).
set -o pipefail
TAG=${1:-c5d}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for T in L E G; do
  timeout -k 10 300 python -u scripts/probes/phase_timing.py --c5 --group64 --types $T --steps 2 --commits 33000000 > $OUT/phase_$T.txt 2>&1 || { echo "phase $T failed"; tail -5 $OUT/phase_$T.txt; exit 1; }
  grep -v "^W2026\|amdgpu.ids" $OUT/phase_$T.txt | head -14
done
timeout -k 10 300 python -u scripts/probes/phase_timing.py --c5 --manager --steps 2 > $OUT/phase_mgr.txt 2>&1 || { echo "phase mgr failed"; tail -5 $OUT/phase_mgr.txt; exit 1; }
grep -v "^W2026\|amdgpu.ids" $OUT/phase_mgr.txt | head -14
for m in new v1; do
  case $m in new) ENVS="";; v1) ENVS="CC_EV_V1=1";; esac
  env $ENVS timeout -k 10 600 python -u bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline --no-parity > $OUT/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 $OUT/bench_$m.log; exit 1; }
  tail -1 $OUT/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$m', d['value']/1e9, d['ms_per_step'], r['per_kernel_ms_per_step'])"
done

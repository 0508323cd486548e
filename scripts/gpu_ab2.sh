#!/bin/bash
# Full GPU test suite + phase clocks + c2 bench, then the c2 bench with each experiment knob in "$@".
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probes/phase_timing.py > $OUT/phase.log 2>&1 || { tail $OUT/phase.log; exit 1; }
grep -v amdgpu.ids $OUT/phase.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200; grep -o '"per_kernel_ms_per_step": {[^}]*}' $OUT/bench.log
for kv in "$@"; do
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$kv.log 2>&1 || { tail $OUT/bench_$kv.log; exit 1; }
  echo "$kv"; tail -1 $OUT/bench_$kv.log | cut -c1-200; grep -o '"per_kernel_ms_per_step": {[^}]*}' $OUT/bench_$kv.log
done
echo all-ok

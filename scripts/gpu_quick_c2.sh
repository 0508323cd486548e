#!/bin/bash
# c2 iteration pass: the value tests per mode, then the c2 bench per mode.
# Usage (via gpurun): bash scripts/gpu_quick_c2.sh TAG [modes...]   modes: v3 v2 (default: v3)
set -o pipefail
TAG=${1:-q}; shift
MODES=${@:-v3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for m in $MODES; do
  case $m in v3) ENVS="";; v2) ENVS="CC_VALUE_V2=1";; esac
  env $ENVS timeout -k 10 600 python -u -m pytest tests/test_gpu_value.py tests/test_gpu_scale.py::test_c2_continued_steps -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$m.log 2>&1; rc=$?
  echo "pytest $m rc=$rc"; tail -2 $OUT/pytest_$m.log
  [ $rc -eq 0 ] || exit $rc
  env $ENVS timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 $OUT/bench_$m.log; exit 1; }
  tail -1 $OUT/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$m', d['value']/1e9, d['ms_per_step'], d['parity']['mismatches'], d['parity']['unwritten'], d['parity']['state_mismatches'], r['per_kernel_ms_per_step'], r['pipeline_frac'])"
done

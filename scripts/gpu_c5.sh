#!/bin/bash
# c5 iteration: the coordination / close / retained GPU tests, then the c5 bench (default, then CC_EV_V1=1 A/B).
set -o pipefail
TAG=${1:-c5}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_coord.py tests/test_gpu_close.py tests/test_gpu_retained.py tests/test_gpu_kats.py tests/test_gpu_scale.py::test_c5_mixed_coordination_10m_rows -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for m in new v1; do
  case $m in new) ENVS="";; v1) ENVS="CC_EV_V1=1";; esac
  env $ENVS timeout -k 10 600 python -u bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 $OUT/bench_$m.log; exit 1; }
  tail -1 $OUT/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$m', d['value']/1e9, d['ms_per_step'], d['parity'], d['config']['expiry'], r['per_kernel_ms_per_step'], r['pipeline_frac'])"
done

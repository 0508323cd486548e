#!/bin/bash
# A/B by environment knob: value parity tests with the new default, then the c2 bench with and without ENV.
# Usage (via gpurun): bash scripts/gpu_ab_env.sh TAG ENVVAR [pytest selection]
set -o pipefail
TAG=$1; EV=$2
SEL=${3:-tests/test_gpu_value.py tests/test_gpu_kats.py tests/test_gpu_snapshot.py}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $SEL -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in new old new; do
  if [ $v = old ]; then E="env $EV=1"; else E=""; fi
  timeout -k 10 300 $E python bench.py --no-cpu-baseline --steps 10 > $OUT/bench_$v.log 2>&1 || { tail $OUT/bench_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,2), d['ms_per_step'], d.get('parity',{}).get('mismatches'), {k: v for k, v in d['roofline']['per_kernel_ms_per_step'].items() if v})"
done
echo all-ok

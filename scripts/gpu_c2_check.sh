#!/bin/bash
# c2 check after a value-path change: value / scale / KAT GPU tests, then a c2 bench line with its full step-0 gate.
# Usage: bash scripts/gpu_c2_check.sh TAG [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-c2c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_value.py tests/test_gpu_scale.py tests/test_gpu_kats.py -x -q --timeout 120 --timeout-method thread -m gpu ${2:+-k "$2"} > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 2 > $OUT/bench_c2.log 2>&1 || { tail $OUT/bench_c2.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c2.log').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']/1e9,3), d['ms_per_step'], d['parity'], r.get('frac'), r.get('per_kernel_ms_per_step'))"
echo all-ok

#!/bin/bash
# c2 check after a value-path change: phase clocks (diagnostics build), value / scale / KAT GPU tests, a c2 bench
# line with its full step-0 gate.  Usage: bash scripts/gpu_c2_quick.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-c2q}
mkdir -p $OUT
export TMPDIR=/tmp
CC_V3_PHASES=1 timeout -k 10 200 python scripts/probes/phase_timing.py --steps 3 > $OUT/phase_c2.txt 2>&1 || { tail $OUT/phase_c2.txt; exit 1; }
grep -v amdgpu.ids $OUT/phase_c2.txt | head -9
timeout -k 10 600 python -u -m pytest tests/test_gpu_value.py tests/test_gpu_scale.py tests/test_gpu_kats.py tests/test_gpu_host_boundary.py -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 2 > $OUT/bench_c2.log 2>&1 || { tail $OUT/bench_c2.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c2.log').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value']/1e9,3), d['ms_per_step'], d['parity']['mismatches'], r.get('pipeline_frac'), r.get('per_kernel_ms_per_step'))"
echo all-ok

#!/bin/bash
# Map / coordination path check: map, coordination and scale GPU tests, then c3 and c5 bench lines with their gates.
# Usage (via gpurun): bash scripts/gpu_c3c5_check.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-c3c5}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_coord.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c3.log 2>&1 || { tail -5 $OUT/bench_c3.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c3.log').read().strip().splitlines()[-1]); print('c3', round(d['value']/1e9,3), d['ms_per_step'], d['parity']['mismatches'], d['parity']['maps_mismatched'], d['roofline']['per_kernel_ms_per_step'])"
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { tail -5 $OUT/bench_c5.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c5.log').read().strip().splitlines()[-1]); print('c5', round(d['value']/1e9,3), d['ms_per_step'], d['parity']['mismatches'], d['parity']['events_equal'], d['roofline']['per_kernel_ms_per_step'])"
echo check-ok

#!/bin/bash
# c5 check after a partition / coordination change: coordination GPU tests and a c5 bench line (no gate).
# Usage: bash scripts/gpu_c5_quick.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-c5q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_coord.py tests/test_gpu_close.py tests/test_gpu_kats.py -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_c5.log 2>&1 || { tail -30 $OUT/pytest_c5.log; exit 1; }
tail -2 $OUT/pytest_c5.log
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-parity --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { tail $OUT/bench_c5.log; exit 1; }
tail -1 $OUT/bench_c5.log | cut -c1-300
echo c5-ok

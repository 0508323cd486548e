#!/bin/bash
# Extended-staging paths after a kernel change: map / coord / retained parity tests, then c5 and c3 bench lines.
# Usage (via gpurun): bash scripts/gpu_ext.sh TAG [pytest selection]
set -o pipefail
TAG=${1:-ext}
SEL=${2:-tests/test_gpu_map.py tests/test_gpu_coord.py tests/test_gpu_kats.py tests/test_gpu_retained.py}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest $SEL -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c5.log 2>&1 || { tail $OUT/c5.log; exit 1; }
python -c "import json; d=json.loads(open('$OUT/c5.log').read().strip().splitlines()[-1]); print('c5', d['value']/1e9, d['ms_per_step'], d['roofline'].get('per_kernel_ms_per_step'))"
timeout -k 10 400 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
python -c "import json; d=json.loads(open('$OUT/c3.log').read().strip().splitlines()[-1]); print('c3', d['value']/1e9, d['ms_per_step'], d['roofline'].get('per_kernel_ms_per_step'))"
echo all-ok

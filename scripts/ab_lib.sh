#!/bin/bash
# A/B of an alternative engine build: bench c2 with the in-tree .so, then with scratch_ab/$1 copied over it.
set -o pipefail
OUT=gpurun_out/ab_lib; mkdir -p $OUT
timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 1; }
python -c "import json; d=json.loads(open('$OUT/a.log').read().strip().splitlines()[-1]); print('A', d['value']/1e9, d['roofline']['per_kernel_ms_per_step'])"
cp scratch_ab/$1 copycat_amd/libcopycat_apply.so
timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
python -c "import json; d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('B', d['value']/1e9, d['roofline']['per_kernel_ms_per_step'])"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_value.py > $OUT/pytest_b.log 2>&1; tail -1 $OUT/pytest_b.log

#!/bin/bash
# Round 4: value-only pipeline with results stored at their log rows (A) vs the unpermute pipeline (B, -DCC_VALUE_UNPERMUTE).
set -o pipefail
OUT=gpurun_out/${1:-ab_direct}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_value.py tests/test_gpu_map.py tests/test_gpu_snapshot.py tests/test_gpu_set.py tests/test_gpu_close.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/a$i.log 2>&1 || { tail $OUT/a$i.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/a$i.log').read().strip().splitlines()[-1]); print('A direct', d['value']/1e9, d['ms_per_step'], d['roofline']['per_kernel_ms_per_step'])"
  CC_ENGINE_SO=copycat_amd/diag/libcopycat_apply_unperm.so timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/b$i.log 2>&1 || { tail $OUT/b$i.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/b$i.log').read().strip().splitlines()[-1]); print('B unperm', d['value']/1e9, d['ms_per_step'], d['roofline']['per_kernel_ms_per_step'])"
done

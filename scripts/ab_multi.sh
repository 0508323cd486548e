#!/bin/bash
# A/B of several alternative engine builds: c2 bench + value parity tests with the in-tree .so, then with each
# scratch_ab/<name>.so copied over it.  Usage (via gpurun): bash scripts/ab_multi.sh name1.so name2.so ...
set -o pipefail
OUT=gpurun_out/ab_multi; mkdir -p $OUT
export TMPDIR=/tmp
cp copycat_amd/libcopycat_apply.so $OUT/base.so.keep
run() {
  timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/$1.log 2>&1 || { tail $OUT/$1.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$1.log').read().strip().splitlines()[-1]); print('$1', d['value']/1e9, d['roofline']['per_kernel_ms_per_step'])"
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_value.py tests/test_gpu_kats.py > $OUT/pytest_$1.log 2>&1 || { echo "pytest $1 failed"; tail $OUT/pytest_$1.log; exit 1; }
  tail -1 $OUT/pytest_$1.log
}
run base
for v in "$@"; do cp scratch_ab/$v copycat_amd/libcopycat_apply.so; run ${v%.so}; done
cp $OUT/base.so.keep copycat_amd/libcopycat_apply.so; rm -f $OUT/base.so.keep
echo all-ok

#!/bin/bash
# A/B of alternative engine builds on the extended-staging workloads (c5, c3): coord/map parity tests with each
# variant, then the c5 and c3 bench lines.  Usage (via gpurun): bash scripts/ab_ext.sh name1.so ...
set -o pipefail
OUT=gpurun_out/ab_ext; mkdir -p $OUT
export TMPDIR=/tmp
cp copycat_amd/libcopycat_apply.so $OUT/base.so.keep
run() {
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_coord.py tests/test_gpu_map.py tests/test_gpu_kats.py > $OUT/pytest_$1.log 2>&1 || { echo "pytest $1 failed"; tail $OUT/pytest_$1.log; exit 1; }
  tail -1 $OUT/pytest_$1.log
  for wl in c5 c3; do
    S=5; [ $wl = c3 ] && S=3
    timeout -k 10 300 python bench.py --workload $wl --steps $S --warmup 1 --no-cpu-baseline --no-parity > $OUT/${1}_$wl.log 2>&1 || { tail $OUT/${1}_$wl.log; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${1}_$wl.log').read().strip().splitlines()[-1]); print('$1 $wl', round(d['value']/1e9,3), d['ms_per_step'], {k: v for k, v in d['roofline']['per_kernel_ms_per_step'].items() if v > 0.1})"
  done
}
run base
for v in "$@"; do cp scratch_ab/$v copycat_amd/libcopycat_apply.so; run ${v%.so}; done
cp $OUT/base.so.keep copycat_amd/libcopycat_apply.so; rm -f $OUT/base.so.keep
echo all-ok

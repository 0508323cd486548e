#!/bin/bash
# A/B of engine variants on c3 / c5 (diagnostics): GPU tests of the map / coordination paths, bench lines per
# library (VARIANTS: main = the in-tree library, X = copycat_amd/diag/libcopycat_apply_X.so), c3 phase table.
set -o pipefail
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_set.py tests/test_gpu_multimap.py tests/test_gpu_coord.py tests/test_gpu_queue.py tests/test_gpu_kats.py tests/test_gpu_snapshot.py tests/test_gpu_retained.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in ${VARIANTS:-main}; do
  if [ $v = main ]; then unset CC_ENGINE_SO; else export CC_ENGINE_SO=$PWD/copycat_amd/diag/libcopycat_apply_$v.so; fi
  for wl in ${WORKLOADS:-c3 c5}; do
    timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/${wl}_$v.log 2>&1 || { tail $OUT/${wl}_$v.log; exit 1; }
    tail -1 $OUT/${wl}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', '$v', round(d['value']/1e9, 3), d['roofline']['per_kernel_ms_per_step'])"
  done
done
unset CC_ENGINE_SO
timeout -k 10 200 python3 scripts/probes/phase_timing.py --c3 --commits 100000000 --steps 2 > $OUT/phase.txt 2>&1; tail -22 $OUT/phase.txt

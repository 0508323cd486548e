#!/bin/bash
# Quick A/B pass: value parity tests, then c2 benches (default and with the experiment knobs in $AB_ENVS).
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_value.py tests/test_gpu_kats.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
for kv in "$@"; do
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$kv.log 2>&1 || { tail $OUT/bench_$kv.log; exit 1; }
  echo "$kv"; tail -1 $OUT/bench_$kv.log
done
echo all-ok

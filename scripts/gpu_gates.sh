#!/bin/bash
# GPU pass: the -m gpu suite, smoke, then every workload's bench line with its parity gate.
# Usage (via gpurun): bash scripts/gpu_gates.sh TAG [workloads...]   (default: c2 c4 c5 c3)
set -o pipefail
TAG=${1:-gates}; shift
WLS=${@:-c2 c4 c5 c3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
fi
for w in $WLS; do
  case $w in
    c2) A="--steps 20 --warmup 2";;
    c3) A="--workload c3 --steps 2 --warmup 1";;
    c4) A="--workload c4 --steps 50 --warmup 5";;
    c5) A="--workload c5 --steps 4 --warmup 1";;
  esac
  timeout -k 10 600 python -u bench.py $A > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-600
done
echo all-ok

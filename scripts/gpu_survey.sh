#!/bin/bash
# One GPU-box pass over every workload: parity tests, smoke, benches (c2 at several sub-batch sizes, c3, c4),
# and a rocprofv3 kernel trace of the default bench.  Usage (via gpurun): bash scripts/gpu_survey.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-survey}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $OUT/progress.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a $OUT/progress.log
  tail -2 $OUT/$name.log
  return $rc
}
if [ "$2" != "skip-tests" ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
step bench_c2 300 python bench.py || exit 1
step bench_c2_sb4m 300 python bench.py --sub-batch 4194304 --no-cpu-baseline || exit 1
step bench_c2_sb2m 300 python bench.py --sub-batch 2097152 --no-cpu-baseline || exit 1
step bench_c3 500 python bench.py --workload c3 --steps 3 --warmup 1 || exit 1
step bench_c4 300 python bench.py --workload c4 || exit 1
step kt_c2 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile || exit 1
echo all-ok

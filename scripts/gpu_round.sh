#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel trace + HBM counters (separate --pmc passes).
# Usage (via gpurun): bash scripts/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BARGS="$@"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py $BARGS > $OUT/bench.log 2>&1 || { echo bench failed; tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $OUT/kt.log 2>&1 || { echo rocprof-kt failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $OUT/fetch.log 2>&1 || { echo rocprof-fetch failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $OUT/write.log 2>&1 || { echo rocprof-write failed; exit 1; }
echo all-ok

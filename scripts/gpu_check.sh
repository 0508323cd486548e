#!/bin/bash
# One GPU-box pass: the whole -m gpu suite, smoke, then the default bench line (c2) with the PCIe-inclusive figure.
# Usage (via gpurun): bash scripts/gpu_check.sh TAG [extra bench args...]
set -o pipefail
TAG=${1:-check}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.log 2>&1 || { echo bench failed; tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
echo all-ok

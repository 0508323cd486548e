#!/bin/bash
# Quick GPU pass after a kernel change: value/map/coord parity tests, phase clocks, c2 bench.
# Usage (via gpurun): bash scripts/gpu_quick.sh TAG [pytest selection]
set -o pipefail
TAG=${1:-quick}
SEL=${2:-tests/test_gpu_value.py tests/test_gpu_kats.py}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $SEL -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probes/phase_timing.py > $OUT/phase.log 2>&1 || { tail $OUT/phase.log; exit 1; }
grep -v amdgpu.ids $OUT/phase.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
echo all-ok

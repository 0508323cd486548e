#!/bin/bash
# k_apply_coord phase clocks per resource type (diagnostics build copycat_amd/diag/libcopycat_apply_phase.so).
set -o pipefail
TAG=${1:-c5p}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for T in ${@:-G E L}; do
  timeout -k 10 300 python -u scripts/probes/phase_timing.py --c5 --group64 --types $T --steps 2 --commits 33000000 > $OUT/phase_$T.txt 2>&1 || { echo "phase $T failed"; tail -5 $OUT/phase_$T.txt; exit 1; }
  grep -v "^W2026\|amdgpu.ids" $OUT/phase_$T.txt | head -9
done

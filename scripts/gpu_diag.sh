#!/bin/bash
# Diagnostics pass: c2 value-path phase clocks (diag build), c5 k_apply_coord phase clocks per type, events A/B.
set -o pipefail
TAG=${1:-diag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CC_V3_PHASES=1 timeout -k 10 300 python -u scripts/probes/phase_timing.py --steps 3 > $OUT/phase_c2.txt 2>&1 || { echo "phase c2 failed"; tail -5 $OUT/phase_c2.txt; exit 1; }
grep -v "^W2026\|amdgpu.ids" $OUT/phase_c2.txt | head -24
bash scripts/gpu_c5_diag.sh $TAG/c5

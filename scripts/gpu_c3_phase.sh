#!/bin/bash
# c3 phase clocks of k_part_ext (CC_PART_EXT_PHASES) and k_apply_map from the diagnostics build, then
# scripts/gpu_c3_quick.sh.  Usage: bash scripts/gpu_c3_phase.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-c3p}
mkdir -p $OUT
export TMPDIR=/tmp
CC_PART_EXT_PHASES=1 timeout -k 10 200 python scripts/probes/phase_timing.py --c3 --steps 2 > $OUT/phase_c3.txt 2>&1 || { tail $OUT/phase_c3.txt; exit 1; }
grep -v amdgpu.ids $OUT/phase_c3.txt | head -24
bash scripts/gpu_c3_quick.sh ${1:-c3p}

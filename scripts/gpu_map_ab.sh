#!/bin/bash
# k_apply_map A/B: phase clocks of the base and current diagnostics builds on the c3 stream, the map parity tests,
# then a c3 bench line.  Usage: bash scripts/gpu_map_ab.sh TAG [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-mapab}
mkdir -p $OUT
export TMPDIR=/tmp
PHASE_SO=copycat_amd/diag/libcopycat_apply_phase_base.so timeout -k 10 200 python scripts/probes/phase_timing.py --c3 --steps 2 > $OUT/phase_base.txt 2>&1 || { tail $OUT/phase_base.txt; exit 1; }
timeout -k 10 200 python scripts/probes/phase_timing.py --c3 --steps 2 > $OUT/phase_new.txt 2>&1 || { tail $OUT/phase_new.txt; exit 1; }
grep -v amdgpu.ids $OUT/phase_base.txt | head -12; grep -v amdgpu.ids $OUT/phase_new.txt | head -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_scale.py tests/test_gpu_set.py tests/test_gpu_multimap.py -x -q --timeout 300 --timeout-method thread -m gpu ${2:+-k "$2"} > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-parity --no-cpu-baseline > $OUT/bench_c3.log 2>&1 || { tail $OUT/bench_c3.log; exit 1; }
tail -1 $OUT/bench_c3.log | cut -c1-300
echo all-ok

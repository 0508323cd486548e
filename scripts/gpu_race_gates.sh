#!/bin/bash
# The small-map replay race-freedom gates (common.h small-map window invariant): the GPU suite, then the
# 1e9-row c3 gate with the default build and with the 1,536-workgroup hot-apply build that exposed the round-5 race
# (built with -DCC_DIAG=4: the replay's snapshot-flag check), plus the whole-map variant on that build.
# Usage (via gpurun): bash scripts/gpu_race_gates.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-race}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c3_default.log 2>&1 || { tail -5 $OUT/c3_default.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3_default.log').read().strip().splitlines()[-1]); print('default', round(d['value']/1e9,3), d['parity']['mismatches'], d['parity']['maps_mismatched'])"
CC_ENGINE_SO=$PWD/copycat_amd/libcopycat_apply_g1536.so timeout -k 10 400 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c3_g1536.log 2>&1 || { tail -5 $OUT/c3_g1536.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3_g1536.log').read().strip().splitlines()[-1]); print('g1536+checks', round(d['value']/1e9,3), d['parity']['mismatches'], d['parity']['maps_mismatched'])"
CC_ENGINE_SO=$PWD/copycat_amd/libcopycat_apply_g1536.so timeout -k 10 400 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --cv-rate 0.001 --clear-rate 0.0001 > $OUT/c3w_g1536.log 2>&1 || { tail -5 $OUT/c3w_g1536.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3w_g1536.log').read().strip().splitlines()[-1]); print('whole-map g1536+checks', round(d['value']/1e9,3), d['parity']['mismatches'], d['parity']['maps_mismatched'])"
echo race-gates-ok

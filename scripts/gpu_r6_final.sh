#!/bin/bash
# Round-6 gates: the GPU suite, smoke, the driver's default bench command (c2 line + c3 sub-record, both gated), then
# profiles (kernel trace + counter passes) of the given workloads.  Usage (via gpurun): bash scripts/gpu_r6_final.sh TAG [c2 c3 ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
T0=$(date +%s)
timeout -k 10 580 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.log 2>&1 || { tail -5 $OUT/bench_default.log; exit 1; }
echo "default bench wall $(( $(date +%s) - T0 )) s"
python3 -c "
import json; d=json.loads(open('$OUT/bench_default.log').read().strip().splitlines()[-1]); c=d['c3']
print('c2', round(d['value']/1e9,3), d['ms_per_step'], d['parity']['mismatches'], d['roofline']['frac'], d['roofline']['traffic_bytes_per_commit'])
print('c3', round(c['value']/1e9,3), c['ms_per_step'], c['parity']['mismatches'], c['parity']['maps_mismatched'], c['roofline']['frac'], c['roofline']['traffic_bytes_per_commit'])"
[ $# -gt 0 ] && bash scripts/gpu_prof_all.sh $TAG "$@"
echo final-ok

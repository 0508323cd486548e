#!/bin/bash
# The c3 barrier variant: 10M rows of c3 with 0.1 % containsValue, 0.01 % clear, plus 0.1 %
# null-valued puts and 0.001 % Delete rows, beside the same rows without the nulls and Deletes (full gates).
# Usage (via gpurun): bash scripts/gpu_c3_barrier_variant.sh TAG [commits]
set -o pipefail
OUT=gpurun_out/${1:-c3b}
N=${2:-10000000}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload c3 --commits $N --steps 1 --warmup 1 --no-cpu-baseline --cv-rate 0.001 --clear-rate 0.0001 > $OUT/c3w.log 2>&1 || { tail -5 $OUT/c3w.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3w.log').read().strip().splitlines()[-1]); print('c3w', round(d['value']/1e9,4), d['ms_per_step'], d['parity']['mismatches'], d['parity']['maps_mismatched'], d['config']['whole_map']['engine_counters'])"
timeout -k 10 600 python bench.py --workload c3 --commits $N --steps 1 --warmup 1 --no-cpu-baseline --cv-rate 0.001 --clear-rate 0.0001 --null-rate 0.001 --delete-rate 0.00001 > $OUT/c3b.log 2>&1 || { tail -5 $OUT/c3b.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3b.log').read().strip().splitlines()[-1]); print('c3b', round(d['value']/1e9,4), d['ms_per_step'], d['parity']['mismatches'], d['parity']['maps_mismatched'], d['config']['whole_map']['engine_counters'])"
echo barrier-variant-ok

#!/bin/bash
# c3 check after a map-path change: map / set / multimap / scale GPU tests, a c3 bench line (no gate), and a kernel
# trace of a 200M-commit c3 run.  Usage: bash scripts/gpu_c3_quick.sh TAG [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-c3q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_scale.py tests/test_gpu_set.py tests/test_gpu_multimap.py -x -q --timeout 300 --timeout-method thread -m gpu ${2:+-k "$2"} > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-parity --no-cpu-baseline > $OUT/bench_c3.log 2>&1 || { tail $OUT/bench_c3.log; exit 1; }
tail -1 $OUT/bench_c3.log | cut -c1-300
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/kt -o run --output-format csv -- python3 $R/bench.py --workload c3 --steps 2 --warmup 1 --commits 200000000 --no-parity --no-cpu-baseline --no-profile --no-e2e > $R/$OUT/kt.log 2>&1 || { tail $R/$OUT/kt.log; exit 1; }
cd $R
STATS=$(find $OUT/kt -name "*kernel_stats.csv" | head -1)
cp $STATS $OUT/kernel_stats.csv
find $OUT/kt -name "*kernel_trace.csv" -delete
python3 -c "
import csv
rows = list(csv.DictReader(open('$OUT/kernel_stats.csv')))
print(f\"{'kernel':44s} {'calls':>6s} {'avg_us':>10s} {'total_ms':>10s}\")
for r in rows:
    n = r['Name'].split('(')[0].replace('void ', '').replace('cc::', '')
    print(f\"{n[:44]:44s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:10.1f} {float(r['TotalDurationNs'])/1e6:10.3f}\")
" > $OUT/kt_summary.txt
head -16 $OUT/kt_summary.txt
echo all-ok

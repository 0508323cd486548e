#!/bin/bash
# c3 (maps, Zipf) and c4 (quorum + expiry) benches plus a kernel trace of c3.  Usage: bash scripts/gpu_c3c4.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-c3c4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --workload c3 --steps 3 --warmup 1 > $OUT/bench_c3.log 2>&1 || { tail $OUT/bench_c3.log; exit 1; }
tail -1 $OUT/bench_c3.log | cut -c1-400
timeout -k 10 300 python bench.py --workload c4 > $OUT/bench_c4.log 2>&1 || { tail $OUT/bench_c4.log; exit 1; }
tail -1 $OUT/bench_c4.log | cut -c1-400
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/kt_c3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $OUT/kt_c3.log 2>&1 || { tail $OUT/kt_c3.log; exit 1; }
echo all-ok

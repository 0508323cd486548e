#!/bin/bash
# rocprofv3 kernel-trace stats of the c4 and c5 bench modes at HEAD.
set -o pipefail
OUT=gpurun_out/kt_modes; mkdir -p $OUT
export TMPDIR=/tmp
for w in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$w -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $OUT/$w.log 2>&1 || { echo "rocprof $w failed"; tail $OUT/$w.log; exit 1; }
  head -8 $OUT/$w/run_kernel_stats.csv | cut -d, -f1-5
done
echo all-ok

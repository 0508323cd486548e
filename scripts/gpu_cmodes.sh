#!/bin/bash
# Bench lines of the non-default workloads (c3 maps, c4 quorum/expiry, c5 coordination) at HEAD.
set -o pipefail
OUT=gpurun_out/cmodes; mkdir -p $OUT
export TMPDIR=/tmp
for w in c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed"; tail $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log > $OUT/bench_$w.json; cut -c1-400 $OUT/bench_$w.json
done
echo all-ok

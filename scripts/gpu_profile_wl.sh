#!/bin/bash
# Kernel trace + HBM counters (separate --pmc passes) of one bench workload, then the per-launch traffic table.
# Usage (via gpurun): bash scripts/gpu_profile_wl.sh TAG WORKLOAD [bench args...]
set -o pipefail
TAG=$1; WL=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --workload $WL --no-cpu-baseline --no-profile --no-parity $@"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/kt -o run --output-format csv -- python3 $B > $GRAFT_REPO_ROOT/$OUT/kt.log 2>&1 || { echo rocprof-kt failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$OUT/fetch -o run --output-format csv -- python3 $B > $GRAFT_REPO_ROOT/$OUT/fetch.log 2>&1 || { echo rocprof-fetch failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$OUT/write -o run --output-format csv -- python3 $B > $GRAFT_REPO_ROOT/$OUT/write.log 2>&1 || { echo rocprof-write failed; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/pmc_traffic.py $OUT $OUT/traffic.json $WL > $OUT/traffic.txt && python3 scripts/prof_summary.py $OUT > $OUT/summary.txt
rm -f $OUT/kt/*kernel_trace.csv
tail -1 $OUT/kt.log | cut -c1-200
echo profile-ok

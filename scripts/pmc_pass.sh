#!/bin/bash
# One rocprofv3 --pmc pass over a short bench run (counters collected alone: no tracing domains combined).
# Usage (via gpurun): bash scripts/pmc_pass.sh OUTDIR "COUNTERS" [bench args...]
set -o pipefail
OUT=$1; CNT=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $CNT -d $GRAFT_REPO_ROOT/$OUT -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-profile --no-parity "$@" > $GRAFT_REPO_ROOT/$OUT/log.txt 2>&1

#!/bin/bash
# Profiles at the bench configs (kernel trace + stats, then FETCH / WRITE / SQ / LDS counter passes), one folder per
# workload under gpurun_out/TAG/prof_<w>, then the whole-step traffic per commit (scripts/pmc_traffic.py).
# Usage (via gpurun): bash scripts/gpu_prof_all.sh TAG c2 c3 c5 c4
set -o pipefail
TAG=$1; shift
for W in "$@"; do
  case $W in
    c2) A="--workload c2 --steps 2 --warmup 1 --no-split"; C=300000000;;
    c3) A="--workload c3 --steps 1 --warmup 1"; C=2000000000;;
    c3w) A="--workload c3 --steps 1 --warmup 1 --cv-rate 0.001 --clear-rate 0.0001"; C=2000000000;;
    c5) A="--workload c5 --steps 2 --warmup 1"; C=300000000;;
    c4) A="--workload c4 --steps 20 --warmup 2"; C=0;;
  esac
  bash scripts/gpu_prof.sh $TAG/prof_$W $A || exit 1
  # (c4: per-launch bytes only -- its units are groups and sessions, not commits)
  if [ $C -gt 0 ]; then python3 scripts/pmc_traffic.py gpurun_out/$TAG/prof_$W gpurun_out/$TAG/traffic.json $W $C > /dev/null || exit 1
  else python3 scripts/pmc_traffic.py gpurun_out/$TAG/prof_$W gpurun_out/$TAG/traffic.json $W > /dev/null || exit 1; fi
done
echo prof-all-ok

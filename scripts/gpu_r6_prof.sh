#!/bin/bash
# Round 6 profiles: the GPU suite, then kernel traces and FETCH / WRITE / SQ / LDS passes of the given workloads
# (scripts/gpu_prof_all.sh) into gpurun_out/TAG.  Usage (via gpurun): bash scripts/gpu_r6_prof.sh TAG c3 c3w c5 c4
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
bash scripts/gpu_prof_all.sh $TAG "$@"

set -o pipefail
mkdir -p gpurun_out/r6b
export TMPDIR=/tmp
T0=$(date +%s)
timeout -k 10 580 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6b/bench_default.log 2>&1 || { tail -5 gpurun_out/r6b/bench_default.log; exit 1; }
echo "default bench wall $(( $(date +%s) - T0 )) s"
bash scripts/gpu_prof_all.sh r6b c2

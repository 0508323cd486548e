set -o pipefail
mkdir -p gpurun_out/c3ph
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c3ph/pytest.log 2>&1 || { tail -20 gpurun_out/c3ph/pytest.log; exit 1; }
tail -1 gpurun_out/c3ph/pytest.log
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c3ph/bench_c3.log 2>&1 || { tail -5 gpurun_out/c3ph/bench_c3.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/c3ph/bench_c3.log').read().strip().splitlines()[-1]); print('c3', round(d['value']/1e9,3), d['ms_per_step'], d['parity']['mismatches'], d['parity']['maps_mismatched'], d['roofline']['per_kernel_ms_per_step'])"
CC_PART_EXT_PHASES=1 PHASE_SO=$PWD/copycat_amd/libcopycat_apply_phase.so timeout -k 10 200 python scripts/probes/phase_timing.py --c3 --commits 200000000 --steps 2 > gpurun_out/c3ph/phase_c3.txt 2>&1; grep -v amdgpu.ids gpurun_out/c3ph/phase_c3.txt | head -30

#!/bin/bash
# Scattering sweep, 4 cells in flight: config-3 parity + bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_golden_r2.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r3d_tests.log | head -30; tail -30 gpurun_out/r3d_tests.log; exit 1; }
tail -1 gpurun_out/r3d_tests.log
timeout -k 10 300 python -u bench.py --config scattering --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r3d_bench_cfg3.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3d_bench_cfg3.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3d_bench_cfg3.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['mean_nfev'], d['roofline']['frac'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
timeout -k 10 300 python -u tools/post_probe.py > gpurun_out/r3d_post.log 2>&1 || { echo "post probe failed"; tail -20 gpurun_out/r3d_post.log; exit 1; }
tail -6 gpurun_out/r3d_post.log
timeout -k 10 300 python -u tools/phase_probe.py 10000 > gpurun_out/r3d_phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/r3d_phase.log; exit 1; }
tail -2 gpurun_out/r3d_phase.log

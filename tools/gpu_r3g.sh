#!/bin/bash
# k_moments / recentring with phasor re-seed every 2 blocks: parity tests + bench (U 8 and 4).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_taylor.py tests/test_gpu_configs.py tests/test_gpu_kernels.py tests/test_gpu_drivers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r3g_tests.log | head -30; tail -30 gpurun_out/r3g_tests.log; exit 1; }
tail -1 gpurun_out/r3g_tests.log
for u in 4 4; do
PPF_MOMENTS_U=$u timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3g_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3g_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3g_bench.log').read().strip().splitlines()[-1])
print('U $u', d['value'], d['ms_per_step'], d['mean_nfev'], d['status_counts'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

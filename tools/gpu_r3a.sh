#!/bin/bash
# Guess (speculative Nelder-Mead rounds): parity tests, bench, phase clocks.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden_r2.py tests/test_gpu_configs.py tests/test_gpu_taylor.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r3a_tests.log | head -30; tail -30 gpurun_out/r3a_tests.log; exit 1; }
tail -2 gpurun_out/r3a_tests.log
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3a_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3a_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3a_bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['status_counts'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
timeout -k 10 300 python -u tools/phase_probe.py 10000 > gpurun_out/r3a_phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/r3a_phase.log; exit 1; }
tail -4 gpurun_out/r3a_phase.log

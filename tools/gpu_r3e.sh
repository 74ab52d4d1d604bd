#!/bin/bash
# Single-wave guess: bitwise A/B against the block guess, parity tests, bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
PPF_GUESS_WAVE=0 timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/ab_block.npz > gpurun_out/r3e_ab0.log 2>&1 || { echo "A failed"; tail -20 gpurun_out/r3e_ab0.log; exit 1; }
timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/ab_wave.npz > gpurun_out/r3e_ab1.log 2>&1 || { echo "B failed"; tail -20 gpurun_out/r3e_ab1.log; exit 1; }
python tools/guess_ab.py gpurun_out/ab_block.npz gpurun_out/ab_wave.npz
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden_r2.py tests/test_gpu_configs.py tests/test_gpu_taylor.py tests/test_gpu_drivers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3e_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r3e_tests.log | head -30; tail -30 gpurun_out/r3e_tests.log; exit 1; }
tail -1 gpurun_out/r3e_tests.log
for g in 0 1; do
PPF_GUESS_WAVE=$g timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3e_bench_$g.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3e_bench_$g.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3e_bench_$g.log').read().strip().splitlines()[-1])
print('wave $g', d['value'], d['ms_per_step'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

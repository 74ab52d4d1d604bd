#!/bin/bash
# k_moments with the v^m-only power table: bitwise vs the previous build, tests, bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/ab_new.npz > gpurun_out/r3f_ab.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r3f_ab.log; exit 1; }
python tools/guess_ab.py tools/ab_ref_tmp.npz gpurun_out/ab_new.npz
timeout -k 10 600 python -u -m pytest tests/test_gpu_taylor.py tests/test_gpu_configs.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r3f_tests.log | head -30; tail -30 gpurun_out/r3f_tests.log; exit 1; }
tail -1 gpurun_out/r3f_tests.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3f_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3f_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3f_bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

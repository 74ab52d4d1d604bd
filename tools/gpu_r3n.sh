#!/bin/bash
# cell sweeps with alternating register sets: full GPU suite + config 3 + headline bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r3n_tests.log | head -30; tail -5 gpurun_out/r3n_tests.log; exit 1; }
tail -1 gpurun_out/r3n_tests.log
for cfg in scattering scattering headline; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r3n_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3n_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3n_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

#!/bin/bash
# HEAD check: full GPU suite, smoke(), headline bench x2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3t_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r3t_tests.log | head -30; tail -5 gpurun_out/r3t_tests.log; exit 1; }
tail -1 gpurun_out/r3t_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3t_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r3t_smoke.log; exit 1; }
tail -1 gpurun_out/r3t_smoke.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3t_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3t_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3t_bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

#!/bin/bash
# split scattering solve: config-3 parity tests + config-3 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2r_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r2r_tests.log | head -20; tail -5 gpurun_out/r2r_tests.log; exit 1; }
tail -1 gpurun_out/r2r_tests.log
timeout -k 10 400 python -u bench.py --config scattering --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r2r_bench_cfg3.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r2r_bench_cfg3.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r2r_bench_cfg3.log").read().strip().splitlines()[-1])
print(d["ms_per_step"], d["mean_nfev"], d["status_counts"], d["roofline"]["kernel_ms_per_step"], d["roofline"]["frac"], d.get("parity_sample"))
PY

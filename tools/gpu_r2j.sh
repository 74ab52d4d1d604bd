#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2v_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r2v_tests.log | head -20; tail -5 gpurun_out/r2v_tests.log; exit 1; }
tail -1 gpurun_out/r2v_tests.log
timeout -k 10 300 python -u tools/post_probe.py > gpurun_out/r2v_probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/r2v_probe.log; exit 1; }
tail -2 gpurun_out/r2v_probe.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r2v_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r2v_bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r2v_bench.log").read().strip().splitlines()[-1])
print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"], d.get("parity_sample"))
PY

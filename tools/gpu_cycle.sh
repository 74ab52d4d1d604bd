#!/bin/bash
# One measure cycle on the GPU box: device tests, phase clocks, headline bench.
# usage: tools/gpu_cycle.sh TAG [pytest target]   (logs: gpurun_out/TAG_*.log)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=${1:-cyc}
TESTS=${2:-tests}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/${T}_tests.log | head -20; tail -5 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u tools/post_probe.py > gpurun_out/${T}_probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/${T}_probe.log; exit 1; }
tail -2 gpurun_out/${T}_probe.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/${T}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.log; exit 1; }
python - "$T" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/%s_bench.log" % sys.argv[1]).read().strip().splitlines()[-1])
print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"], d.get("parity_sample"))
PY

#!/bin/bash
# Round-3 measure cycle: GPU suite, the solver-trajectory tests verbose,
# headline bench (no legs).  usage: tools/gpu_r3.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver_traj.py -m gpu -q -s --timeout 120 --timeout-method thread > gpurun_out/${T}_traj.log 2>&1 || [ $? -eq 1 ] || { echo "traj tests crashed"; exit 1; }
grep -E "nfev|end point|extra" gpurun_out/${T}_traj.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-legs > gpurun_out/${T}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.log; exit 1; }
python3 - "$T" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/%s_bench.log" % sys.argv[1]).read().strip().splitlines()[-1])
print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])
PY

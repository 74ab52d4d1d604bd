#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2t_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r2t_tests.log; exit 1; }
tail -1 gpurun_out/r2t_tests.log
timeout -k 10 400 python -u bench.py --config gm --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r2t_bench_cfg4.log 2>&1 || { echo "bench failed"; tail -8 gpurun_out/r2t_bench_cfg4.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r2t_bench_cfg4.log").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["host_stream"])
PY

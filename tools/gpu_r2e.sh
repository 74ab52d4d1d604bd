#!/bin/bash
# round-2 GPU pass e: moment-table parity + moments steps-in-flight sweep
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_taylor.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2g_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r2g_tests.log; exit 1; }
tail -2 gpurun_out/r2g_tests.log
for u in 8 4; do
  PPF_MOMENTS_U=$u timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r2g_bench_u$u.log 2>&1 || { echo "bench u=$u failed"; tail -5 gpurun_out/r2g_bench_u$u.log; exit 1; }
  echo "U=$u"; python - "$u" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r2g_bench_u%s.log" % sys.argv[1]).read().strip().splitlines()[-1])
print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"], d.get("parity_sample"))
PY
done

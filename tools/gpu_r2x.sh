#!/bin/bash
# Templates (spline, instrumental response), pipeline bitwise test, then the
# headline bench at 1/2/4/8 pipeline pieces.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_templates.py tests/test_gpu_psrfits.py tests/test_gpu_drivers.py "tests/test_gpu_taylor.py::test_pipeline_pieces_bitwise" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2x_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r2x_tests.log | head -30; tail -40 gpurun_out/r2x_tests.log; exit 1; }
tail -3 gpurun_out/r2x_tests.log
for p in 1 2 4 8; do
  PPF_PIPE=$p timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r2x_bench_p$p.log 2>&1 || { echo "bench $p failed"; tail -5 gpurun_out/r2x_bench_p$p.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/r2x_bench_p$p.log').read().strip().splitlines()[-1])
print('pipe $p', d['value'], d['ms_per_step'], d['status_counts'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

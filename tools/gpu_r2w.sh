#!/bin/bash
# Template producers (spline, instrumental response) + driver regression on the GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_templates.py tests/test_gpu_drivers.py tests/test_gpu_models.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2w_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r2w_tests.log | head -30; tail -40 gpurun_out/r2w_tests.log; exit 1; }
tail -3 gpurun_out/r2w_tests.log

#!/bin/bash
# Newton-CG on the device: golden + oracle cases, then the r2 golden file.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_golden_r2.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r2y_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert|Newton" gpurun_out/r2y_tests.log | head -30; tail -30 gpurun_out/r2y_tests.log; exit 1; }
grep -E "Newton|passed|failed" gpurun_out/r2y_tests.log | tail -12

#!/bin/bash
# round-2 GPU pass d: narrowband TOAs and channel zapping against the reference
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "narrowband or zap" -v -x --timeout 240 --timeout-method thread > gpurun_out/r2d_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r2d_tests.log | tail -30
exit $rc

#!/bin/bash
# round-2 GPU pass b: TNC + golden r2 + configs (with prints), then a short bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden_r2.py tests/test_gpu_configs.py -m gpu -v -s --timeout 300 --timeout-method thread -rf > gpurun_out/r2b_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASS|FAIL|Error|TNC|legacy|headline|nfev" gpurun_out/r2b_tests.log | tail -40
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r2b_bench.log 2>&1
  echo "bench rc=$?"
  tail -1 gpurun_out/r2b_bench.log | cut -c1-1500
fi

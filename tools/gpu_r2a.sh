#!/bin/bash
# round-2 GPU pass: full -m gpu suite, then a short headline bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/r2a_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/r2a_tests.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r2a_bench.log 2>&1
  echo "bench rc=$?"
  tail -3 gpurun_out/r2a_bench.log
fi

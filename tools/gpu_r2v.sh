#!/bin/bash
# Round-2 re-entry gate: full GPU parity suite, headline bench, kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2v_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r2v_tests.log | head -30; tail -5 gpurun_out/r2v_tests.log; exit 1; }
tail -1 gpurun_out/r2v_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r2v_bench.log 2>&1 || { echo "bench failed"; tail -8 gpurun_out/r2v_bench.log; exit 1; }
tail -c 600 gpurun_out/r2v_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2v_prof -o run -- python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r2v_prof.log 2>&1 || { echo "prof failed"; tail -8 gpurun_out/r2v_prof.log; exit 1; }
find gpurun_out/r2v_prof -name '*kernel_stats.csv' | head -3

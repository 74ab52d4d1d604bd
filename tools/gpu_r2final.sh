#!/bin/bash
# Round-2 final evidence: full GPU parity suite, kernel trace + PMC traffic of
# the headline bench, headline / config 3 / config 4 bench lines with CPU baselines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/fin_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/fin_tests.log | head -30; tail -5 gpurun_out/fin_tests.log; exit 1; }
tail -1 gpurun_out/fin_tests.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fin -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 > $R/gpurun_out/prof_fin.log 2>&1 || { echo "kernel trace failed"; tail -5 $R/gpurun_out/prof_fin.log; exit 1; }
echo TRACE_DONE
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_fin -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_fetch_fin.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_fin -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_write_fin.log 2>&1 || { echo "write pass failed"; exit 1; }
echo TRAFFIC_DONE
cd $R
timeout -k 10 400 python -u bench.py > gpurun_out/fin_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/fin_bench.log; exit 1; }
tail -1 gpurun_out/fin_bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py --config scattering --steps 3 --warmup 1 > gpurun_out/fin_bench_cfg3.log 2>&1 || { echo "cfg3 bench failed"; exit 1; }
timeout -k 10 400 python -u bench.py --config gm --steps 3 --warmup 1 > gpurun_out/fin_bench_cfg4.log 2>&1 || { echo "cfg4 bench failed"; exit 1; }
echo BENCH_DONE

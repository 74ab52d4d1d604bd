#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the headline bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-timing > $R/gpurun_out/prof_r1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_r1 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_fetch_r1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_r1 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_write_r1.log 2>&1
echo PROFILE_DONE

#!/bin/bash
# One rocprofv3 counter pass over a short headline bench: pmc_pass.sh TAG "COUNTERS..."
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc $1 -d $R/gpurun_out/pmc_${tag} -o run --output-format csv -- python3 $R/bench.py --nsub 2000 --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_${tag}.log 2>&1 || { echo "pass $tag failed"; tail -5 $R/gpurun_out/pmc_${tag}.log; exit 1; }
python3 $R/tools/pmc_table.py $(find $R/gpurun_out/pmc_${tag} -name "*counter_collection.csv")

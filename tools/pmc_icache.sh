#!/bin/bash
# Counter list + an instruction-cache pass over a short headline bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-ic}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || echo "list failed"
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" $R/gpurun_out/counters_list.txt | sort -u > $R/gpurun_out/counters_sq.txt || true
set1=${2:-"SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH"}
timeout -s KILL 120 rocprofv3 --pmc $set1 -d $R/gpurun_out/pmc_${tag}_1 -o run --output-format csv -- python3 $R/bench.py --nsub 2000 --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_${tag}_1.log 2>&1 || { echo "pass failed"; tail -5 $R/gpurun_out/pmc_${tag}_1.log; }
echo PMC_DONE

#!/bin/bash
# rocprofv3 kernel trace + stats of a short headline bench. Usage: tools/profile_quick.sh tag
set -e
tag=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 > $R/gpurun_out/prof_$tag.log 2>&1
find $R/gpurun_out/prof_$tag -name "*kernel_stats.csv" -exec cat {} \;

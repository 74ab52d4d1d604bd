#!/bin/bash
# Round-1 measurement set for the headline bench: default bench line (with CPU
# baseline), rocprofv3 kernel stats, and separate FETCH_SIZE / WRITE_SIZE passes.
# usage: tools/profile_r1b.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r1b}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 -u $R/bench.py > $O/${tag}_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/${tag}_bench.log; exit 1; }
tail -c 3000 $O/${tag}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${tag}_prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-timing > $O/${tag}_prof.log 2>&1 || { echo "kernel trace failed"; tail -20 $O/${tag}_prof.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/${tag}_fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $O/${tag}_fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 $O/${tag}_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/${tag}_write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $O/${tag}_write.log 2>&1 || { echo "write pass failed"; tail -5 $O/${tag}_write.log; exit 1; }
echo PROFILE_DONE

#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/post_probe.py > gpurun_out/r2i_probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/r2i_probe.log; exit 1; }
cat gpurun_out/r2i_probe.log | tail -3

#!/bin/bash
# config 3 bench line with its CPU baseline (profiles refresh after the cell-sweep change)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config scattering --steps 3 --warmup 1 > gpurun_out/r3p_cfg3.log 2>&1 || { echo "cfg3 bench failed"; tail -5 gpurun_out/r3p_cfg3.log; exit 1; }
tail -1 gpurun_out/r3p_cfg3.log | cut -c1-200

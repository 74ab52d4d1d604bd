#!/bin/bash
# Phase clocks of the latency-bound kernels (guess, fit_taylor, post).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/phase_probe.py 10000 > gpurun_out/r2z_phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/r2z_phase.log; exit 1; }
cat gpurun_out/r2z_phase.log
timeout -k 10 300 python -u tools/post_probe.py > gpurun_out/r2z_post.log 2>&1 || { echo "post probe failed"; tail -20 gpurun_out/r2z_post.log; exit 1; }
tail -8 gpurun_out/r2z_post.log

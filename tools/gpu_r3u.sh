#!/bin/bash
# k_guess_w fold loads four in flight (g1) vs in-tree: bitwise fit outputs + kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
M2=$R/pulseportraiture_amd/libppfit_g1.so
timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3u_def.npz > gpurun_out/r3u_ab_def.log 2>&1 || { echo "ab default failed"; tail -5 gpurun_out/r3u_ab_def.log; exit 1; }
PPF_LIB=$M2 timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3u_g1.npz > gpurun_out/r3u_ab_g1.log 2>&1 || { echo "ab g1 failed"; tail -5 gpurun_out/r3u_ab_g1.log; exit 1; }
python tools/guess_ab.py gpurun_out/r3u_def.npz gpurun_out/r3u_g1.npz
bash tools/gpu_variants.sh r3u default pulseportraiture_amd/libppfit_g1.so default pulseportraiture_amd/libppfit_g1.so

#!/bin/bash
# unpredicated moment loads (m2: k_moments tile16 + recentring tile8) vs in-tree: bitwise fit outputs + kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
M2=$R/pulseportraiture_amd/libppfit_m2.so
timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3s_def.npz > gpurun_out/r3s_ab_def.log 2>&1 || { echo "ab default failed"; tail -5 gpurun_out/r3s_ab_def.log; exit 1; }
PPF_LIB=$M2 timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3s_m2.npz > gpurun_out/r3s_ab_m2.log 2>&1 || { echo "ab m2 failed"; tail -5 gpurun_out/r3s_ab_m2.log; exit 1; }
python tools/guess_ab.py gpurun_out/r3s_def.npz gpurun_out/r3s_m2.npz
bash tools/gpu_variants.sh r3s default pulseportraiture_amd/libppfit_m2.so default pulseportraiture_amd/libppfit_m2.so

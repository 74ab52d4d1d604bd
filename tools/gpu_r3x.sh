#!/bin/bash
# k_fit_taylor at two waves per SIMD without spills (t2) vs in-tree: bitwise fit outputs + kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
M2=$R/pulseportraiture_amd/libppfit_t2.so
timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3x_def.npz > gpurun_out/r3x_ab_def.log 2>&1 || { echo "ab default failed"; tail -5 gpurun_out/r3x_ab_def.log; exit 1; }
PPF_LIB=$M2 timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3x_t2.npz > gpurun_out/r3x_ab_t2.log 2>&1 || { echo "ab t2 failed"; tail -5 gpurun_out/r3x_ab_t2.log; exit 1; }
python tools/guess_ab.py gpurun_out/r3x_def.npz gpurun_out/r3x_t2.npz
bash tools/gpu_variants.sh r3x default pulseportraiture_amd/libppfit_t2.so default pulseportraiture_amd/libppfit_t2.so

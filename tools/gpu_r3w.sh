#!/bin/bash
# k_moments at four waves per SIMD (o4) vs in-tree: bitwise fit outputs + kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
M2=$R/pulseportraiture_amd/libppfit_o4.so
timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3w_def.npz > gpurun_out/r3w_ab_def.log 2>&1 || { echo "ab default failed"; tail -5 gpurun_out/r3w_ab_def.log; exit 1; }
PPF_LIB=$M2 timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3w_o4.npz > gpurun_out/r3w_ab_o4.log 2>&1 || { echo "ab o4 failed"; tail -5 gpurun_out/r3w_ab_o4.log; exit 1; }
python tools/guess_ab.py gpurun_out/r3w_def.npz gpurun_out/r3w_o4.npz
bash tools/gpu_variants.sh r3w default pulseportraiture_amd/libppfit_o4.so default pulseportraiture_amd/libppfit_o4.so

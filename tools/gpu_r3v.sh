#!/bin/bash
# xspec barrier deferred into the next FFT (d1) vs in-tree: bitwise fit outputs + kernel times
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
M2=$R/pulseportraiture_amd/libppfit_d1.so
timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3v_def.npz > gpurun_out/r3v_ab_def.log 2>&1 || { echo "ab default failed"; tail -5 gpurun_out/r3v_ab_def.log; exit 1; }
PPF_LIB=$M2 timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3v_d1.npz > gpurun_out/r3v_ab_d1.log 2>&1 || { echo "ab d1 failed"; tail -5 gpurun_out/r3v_ab_d1.log; exit 1; }
python tools/guess_ab.py gpurun_out/r3v_def.npz gpurun_out/r3v_d1.npz
bash tools/gpu_variants.sh r3v default pulseportraiture_amd/libppfit_d1.so default pulseportraiture_amd/libppfit_d1.so

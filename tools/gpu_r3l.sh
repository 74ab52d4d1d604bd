#!/bin/bash
# k_data_xspec variants: v1 scalar wave index, v3 + branch-free pair loop with alternating template registers
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
bash tools/gpu_variants.sh r3l default pulseportraiture_amd/libppfit_v1.so pulseportraiture_amd/libppfit_v3.so default pulseportraiture_amd/libppfit_v3.so

#!/bin/bash
# k_data_xspec: next row issued after the last template loads (x4) vs in-tree
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
bash tools/gpu_variants.sh r3q default pulseportraiture_amd/libppfit_x4.so default pulseportraiture_amd/libppfit_x4.so

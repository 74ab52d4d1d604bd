#!/bin/bash
# Build the current sources as pulseportraiture_amd/libppfit_$1.so (timing A/B via PPF_LIB).
cd "$(dirname "$0")/.." || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude \
  -Ipulseportraiture_amd/csrc "${@:2}" pulseportraiture_amd/csrc/ppfit_lib.hip \
  -o pulseportraiture_amd/libppfit_$1.so 2>&1 | grep -v "warning\|launch_bounds\|\^\|^ *|" 
ls -la pulseportraiture_amd/libppfit_$1.so

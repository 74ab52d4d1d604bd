#!/bin/bash
# k_moments with unpredicated loads (m1, U=4 and U=8) vs in-tree
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
for v in default m1 m1u8; do
  case $v in default) L=""; U=4;; m1) L="$R/pulseportraiture_amd/libppfit_m1.so"; U=4;; m1u8) L="$R/pulseportraiture_amd/libppfit_m1.so"; U=8;; esac
  PPF_MOMENTS_U=$U PPF_LIB=$L timeout -k 10 200 python -u tools/xspec_probe.py > gpurun_out/r3r_$v.log 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/r3r_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r3r_$v.log)"
done
done

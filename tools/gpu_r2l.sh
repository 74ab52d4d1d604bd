#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for v in default gpurun_nt.so gpurun_m1.so gpurun_ntm1.so; do
  if [ "$v" = default ]; then L=""; else L="$R/$v"; fi
  PPF_LIB=$L timeout -k 10 200 python -u tools/xspec_probe.py > gpurun_out/r2m_$v.log 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/r2l_$v.log; exit 1; }
  tail -1 gpurun_out/r2m_$v.log
done

#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for v in 1 0; do
  PPF_SCAT_SPLIT=$v timeout -k 10 200 python -u tools/cfg3_debug.py > gpurun_out/r2p_$v.log 2>&1 || { echo "debug $v failed"; tail -5 gpurun_out/r2p_$v.log; exit 1; }
  echo "split=$v"; grep -v amdgpu.ids gpurun_out/r2p_$v.log
done

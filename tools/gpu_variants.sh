#!/bin/bash
# Kernel times of alternative builds (PPF_LIB) on the headline batch.
# usage: tools/gpu_variants.sh TAG lib1.so lib2.so ...   ("default" = in-tree)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = default ]; then L=""; else L="$R/$v"; fi
  PPF_LIB=$L timeout -k 10 200 python -u tools/xspec_probe.py > gpurun_out/${T}_$(basename $v).log 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/${T}_$(basename $v).log; exit 1; }
  tail -1 gpurun_out/${T}_$(basename $v).log
done

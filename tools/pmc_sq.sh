#!/bin/bash
# SQ counter passes over a short headline bench (one pass per counter set).
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-sq}
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY" \
           "SQ_INSTS_SALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_${tag}_$i -o run --output-format csv -- python3 $R/bench.py --nsub 2000 --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_${tag}_$i.log; }
done
echo PMC_DONE

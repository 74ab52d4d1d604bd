#!/bin/bash
# Round-4 profile set at HEAD, one config per call:
#   tools/profile_r04.sh TAG CONFIG [NSUB_PMC]
# 1. bench line (HIP-event kernel times, caller legs), 2. rocprofv3
# --kernel-trace --stats of the headline alone (--no-legs), 3. separate --pmc passes: FETCH_SIZE, WRITE_SIZE and
# three SQ sets (instruction mix, waits, LDS, fp64 VALU / MFMA).
# Every GPU step has its own time limit; the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04}
CFG=${2:-headline}
NP=${3:-2000}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
B="$R/bench.py --config $CFG"
timeout -k 10 400 python3 $B --steps 5 --warmup 2 --cpu-sample 0 > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B --steps 5 --warmup 2 --cpu-sample 0 --no-legs > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec head -8 {} \;
pmc() {  # pmc NAME "COUNTERS" NSUB
  timeout -s KILL 150 rocprofv3 --pmc $2 -d $O/pmc_$1 -o run --output-format csv -- python3 $B --nsub $3 --steps 1 --warmup 0 --cpu-sample 0 --no-timing --no-legs > $O/pmc_$1.log 2>&1 || { echo "pmc $1 failed"; tail -3 $O/pmc_$1.log; return 1; }
  echo "pmc $1 ok"
}
NF=${4:-0}
[ "$NF" = "0" ] && NF=$(case $CFG in headline) echo 10000;; gm) echo 2000;; ppalign) echo 1024;; *) echo 1000;; esac)
pmc fetch FETCH_SIZE $NF || exit 1
pmc write WRITE_SIZE $NF || exit 1
python3 $R/tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $NF $O/pmc_traffic_$CFG.json "$T $CFG: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, nsub $NF" || exit 1
pmc sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" $NP || exit 1
pmc sq2 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD" $NP || exit 1
pmc sq3 "SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F64" $NP
echo PROFILE_DONE

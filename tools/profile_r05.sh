#!/bin/bash
# Round-5 profile set at HEAD, one config per call:
#   tools/profile_r05.sh TAG CONFIG [NSUB_PMC] [SQ]
# 1. bench line, 2. rocprofv3 --kernel-trace --stats of the same bench
# command (--no-legs), 3. separate --pmc passes FETCH_SIZE and WRITE_SIZE ->
# pmc_traffic_CONFIG.json (tools/pmc_summary.py), 4. with SQ=1 three SQ sets
# (instruction mix, waits, fp64 VALU / MFMA).  Every GPU step has its own
# time limit; the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r05}
CFG=${2:-headline}
NF=${3:-0}
SQ=${4:-0}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
B="$R/bench.py --config $CFG"
case $CFG in ppalign) RUN="--cpu-sample 0";; *) RUN="--steps 10 --warmup 2 --cpu-sample 0";; esac
timeout -k 10 400 python3 $B $RUN > $O/bench_$CFG.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$CFG.log; exit 1; }
tail -c 300 $O/bench_$CFG.log
LEGS="--no-legs"; [ $CFG = ppalign ] && LEGS=""
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_$CFG -o run --output-format csv -- python3 $B $RUN $LEGS > $O/trace_$CFG.log 2>&1 || { echo "trace failed"; tail -5 $O/trace_$CFG.log; exit 1; }
find $O/trace_$CFG -name "*kernel_stats.csv" -exec head -6 {} \;
[ "$NF" = "0" ] && NF=$(case $CFG in headline) echo 10000;; gm) echo 2000;; ppalign) echo 4096;; *) echo 1000;; esac)
pmc() {  # pmc NAME "COUNTERS"
  case $CFG in ppalign) P="--nsub $NF --cpu-sample 0";; *) P="--nsub $NF --steps 1 --warmup 0 --cpu-sample 0 --no-timing --no-legs";; esac
  timeout -s KILL 200 rocprofv3 --pmc $2 -d $O/pmc_${CFG}_$1 -o run --output-format csv -- python3 $B $P > $O/pmc_${CFG}_$1.log 2>&1 || { echo "pmc $1 failed"; tail -3 $O/pmc_${CFG}_$1.log; return 1; }
  echo "pmc $1 ok"
}
pmc fetch FETCH_SIZE || exit 1
pmc write WRITE_SIZE || exit 1
python3 $R/tools/pmc_summary.py $O/pmc_${CFG}_fetch $O/pmc_${CFG}_write $NF $O/pmc_traffic_$CFG.json "$T $CFG: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, nsub $NF" || exit 1
if [ "$SQ" = "1" ]; then
  pmc sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" || exit 1
  pmc sq2 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_WR" || exit 1
  pmc sq3 "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" || exit 1
fi
echo PROFILE_DONE

#!/bin/bash
# round-2 GPU pass c: TNC tests, rocprof kernel trace + PMC (traffic, SQ) of the
# headline bench, config-3/4 bench lines with CPU baselines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden_r2.py -m gpu -k "tnc" -v -s --timeout 300 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1
echo "pytest rc=$?"; grep -E "PASS|FAIL|TNC|legacy" gpurun_out/r2c_tests.log | tail -12
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r2 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-timing > $R/gpurun_out/prof_r2.log 2>&1 || { echo "kernel trace failed"; exit 1; }
echo TRACE_DONE
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_r2 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_fetch_r2.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_r2 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_write_r2.log 2>&1 || { echo "write pass failed"; exit 1; }
echo TRAFFIC_DONE
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY" \
           "SQ_INSTS_SALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_sq_r2_$i -o run --output-format csv -- python3 $R/bench.py --nsub 2000 --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_sq_r2_$i.log 2>&1 || { echo "sq pass $i failed"; exit 1; }
done
echo SQ_DONE
cd $R
timeout -k 10 400 python -u bench.py --config scattering --steps 3 --warmup 1 > gpurun_out/r2c_bench_cfg3.log 2>&1 || { echo "cfg3 bench failed"; exit 1; }
timeout -k 10 400 python -u bench.py --config gm --steps 3 --warmup 1 > gpurun_out/r2c_bench_cfg4.log 2>&1 || { echo "cfg4 bench failed"; exit 1; }
echo BENCH_DONE

#!/bin/bash
# round-2 GPU pass f: Taylor parity, headline bench, SQ counters of the moment pass
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_taylor.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r2f_tests.log; exit 1; }
tail -1 gpurun_out/r2f_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r2f_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r2f_bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r2f_bench.log").read().strip().splitlines()[-1])
print(d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])
PY
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $R/gpurun_out/pmc_r2f -o run --output-format csv -- python3 $R/bench.py --nsub 2000 --steps 1 --warmup 0 --cpu-sample 0 --no-timing > $R/gpurun_out/pmc_r2f.log 2>&1 || { echo "pmc pass failed"; tail -5 $R/gpurun_out/pmc_r2f.log; exit 1; }
echo PMC_DONE

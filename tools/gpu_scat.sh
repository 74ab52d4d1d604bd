#!/bin/bash
# Scattering-path gate: the GPU tests, then the config-3 bench line.
mkdir -p gpurun_out
tag=${1:-sc}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_all.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_all.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/${tag}_all.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --config scattering --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/${tag}_bench.log 2>&1 || exit 1
python - <<PY
import json; d=json.loads(open("gpurun_out/${tag}_bench.log").read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["mean_nfev"], d["roofline"]["kernel_ms_per_step"])
PY

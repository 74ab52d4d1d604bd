#!/bin/bash
# GPU gate: parity tests then a short bench. Usage: tools/gpu_check.sh [tag] [bench args...]
tag=${1:-check}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_pytest.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${tag}_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 "$@" > gpurun_out/${tag}_bench.log 2>&1
rc=$?
tail -c 1500 gpurun_out/${tag}_bench.log
exit $rc

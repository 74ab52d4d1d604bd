#!/bin/bash
# Quick GPU gate: the whole -m gpu suite, then a short bench line.
mkdir -p gpurun_out
tag=${1:-q}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_all.log 2>&1
rc=$?; tail -5 gpurun_out/${tag}_all.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/${tag}_all.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/${tag}_bench.log 2>&1
rc=$?; tail -c 1200 gpurun_out/${tag}_bench.log; exit $rc

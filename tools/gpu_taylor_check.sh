#!/bin/bash
# GPU gate for the Taylor path: its tests, the whole -m gpu suite, a short bench.
mkdir -p gpurun_out
tag=${1:-t1}
timeout -k 10 300 python -u -m pytest tests/test_gpu_taylor.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_taylor.log 2>&1
rc=$?; tail -25 gpurun_out/${tag}_taylor.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_all.log 2>&1
rc=$?; tail -5 gpurun_out/${tag}_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/${tag}_bench.log 2>&1
rc=$?; tail -c 2500 gpurun_out/${tag}_bench.log; exit $rc

#!/bin/bash
# Bench lines of BASELINE configs 3 and 4 (parity-test shapes, not the headline).
mkdir -p gpurun_out
for c in scattering gm; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/cfg_$c.log 2>&1 || { tail -20 gpurun_out/cfg_$c.log; exit 1; }
  tail -n 1 gpurun_out/cfg_$c.log | cut -c1-400
done

#!/bin/bash
# A/B: moment phasor re-seed every 8 (libppfit.so) vs 16 steps (libppfit_post4.so).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for lib in libppfit.so libppfit_post4.so libppfit.so libppfit_post4.so; do
PPF_LIB=$R/pulseportraiture_amd/$lib timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3i_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3i_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3i_bench.log').read().strip().splitlines()[-1])
print('$lib', d['value'], d['ms_per_step'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

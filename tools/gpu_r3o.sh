#!/bin/bash
# k_scat_sweep at 3 waves/SIMD (168-VGPR cap, spills) vs the in-tree build: config 3 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for v in default pulseportraiture_amd/libppfit_s3.so default pulseportraiture_amd/libppfit_s3.so; do
  if [ "$v" = default ]; then L=""; else L="$R/$v"; fi
  PPF_LIB=$L timeout -k 10 300 python -u bench.py --config scattering --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r3o_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3o_bench.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/r3o_bench.log').read().strip().splitlines()[-1])
print('$(basename $v)', d['value'], d['ms_per_step'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

#!/bin/bash
# k_moments steps in flight: U=8 (default, 168 VGPRs, spills) vs U=4 (140, none).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for u in 8 4 8 4; do
  PPF_MOMENTS_U=$u timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3b_bench_u$u.log 2>&1 || { echo "bench $u failed"; tail -5 gpurun_out/r3b_bench_u$u.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/r3b_bench_u$u.log').read().strip().splitlines()[-1])
print('U $u', d['value'], d['ms_per_step'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

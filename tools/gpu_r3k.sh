#!/bin/bash
# k_moments<2> at 4 waves/SIMD vs k_moments<4> at 3: bitwise A/B of fit outputs + bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for u in 4 2; do
PPF_MOMENTS_U=$u timeout -k 10 200 python -u tools/guess_ab.py gpurun_out/r3k_u$u.npz > gpurun_out/r3k_ab_u$u.log 2>&1 || { echo "ab $u failed"; tail -5 gpurun_out/r3k_ab_u$u.log; exit 1; }
done
python tools/guess_ab.py gpurun_out/r3k_u4.npz gpurun_out/r3k_u2.npz
for u in 4 2 4 2; do
PPF_MOMENTS_U=$u timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3k_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3k_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3k_bench.log').read().strip().splitlines()[-1])
print('U $u', d['value'], d['ms_per_step'], d['mean_nfev'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done

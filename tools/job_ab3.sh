set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab3
for v in c1 dspnt dspnt4 c1 dspnt; do
  PPF_LIB=$R/pulseportraiture_amd/variants/libppfit_$v.so timeout -k 10 300 python3 -u bench.py --config ppalign --cpu-sample 0 > gpurun_out/ab3/pa_$v.json 2> gpurun_out/ab3/pa_$v.err || { echo "ppalign $v failed"; tail -5 gpurun_out/ab3/pa_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab3/pa_$v.json').read().strip().splitlines()[-1]); r=d['detail']
print('ppalign $v', r['ms_per_iteration'], r['kernel_ms_per_iteration']['fit_taylor'])"
done
BENCH_ARGS="--config gm --steps 10 --warmup 2" bash tools/ab_bench.sh ab3gm c1 momu8 c1 momu8 || exit 1
BENCH_ARGS="--steps 10 --warmup 2" bash tools/ab_bench.sh ab3hl c1 momu8 c1 momu8 || exit 1
timeout -k 10 400 python3 -u bench.py --config gm_shard_host --nsub 20000 --shard-chunk 8192 > gpurun_out/ab3/gsh.json 2> gpurun_out/ab3/gsh.err || { echo "gm_shard_host failed"; tail -20 gpurun_out/ab3/gsh.err; exit 1; }
tail -c 1500 gpurun_out/ab3/gsh.json

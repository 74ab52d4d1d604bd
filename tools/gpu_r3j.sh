#!/bin/bash
# bench with pinned async result copies, headline x2 + config 4
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r3j_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3j_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3j_bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['mean_nfev'], d['status_counts'], {k: round(v,3) for k,v in d['roofline']['kernel_ms_per_step'].items()})"
done
timeout -k 10 300 python -u bench.py --config gm --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r3j_cfg4.log 2>&1 || { echo "cfg4 failed"; tail -5 gpurun_out/r3j_cfg4.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3j_cfg4.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['host_stream'])"

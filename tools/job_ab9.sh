set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab9
for v in c1 rot5000 rot20000 rot60000 c1 rot20000; do
  PPF_LIB=$R/pulseportraiture_amd/variants/libppfit_$v.so timeout -k 10 300 python3 -u bench.py --config ppalign --cpu-sample 0 > gpurun_out/ab9/pa_$v.json 2> gpurun_out/ab9/pa_$v.err || { echo "ppalign $v failed"; tail -5 gpurun_out/ab9/pa_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab9/pa_$v.json').read().strip().splitlines()[-1]); r=d['detail']
print('ppalign $v', r['ms_per_iteration'], r['kernel_ms_per_iteration']['fit_taylor'], r['template_finite'])"
done
bash tools/pmc_traffic.sh ab9 ppalign 4096 rot20000

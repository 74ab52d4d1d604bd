set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/ab_variants.sh ab10 headline 10000 tree solo || exit 1
bash tools/ab_variants.sh ab10 gm 2000 tree solo || exit 1
for v in c2 solo c2 solo; do
  PPF_LIB=$R/pulseportraiture_amd/variants/libppfit_$v.so timeout -k 10 300 python3 -u bench.py --config ppalign --cpu-sample 0 > gpurun_out/ab10/pa_$v.json 2> gpurun_out/ab10/pa_$v.err || { echo "ppalign $v failed"; tail -5 gpurun_out/ab10/pa_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab10/pa_$v.json').read().strip().splitlines()[-1]); r=d['detail']
print('ppalign $v', r['ms_per_iteration'], r['kernel_ms_per_iteration']['fit_taylor'])"
done

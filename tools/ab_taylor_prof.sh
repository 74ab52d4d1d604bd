# A/B of the headline step: the in-tree libppfit.so against alt/$1 (built
# beside it from a variant source tree), alternating, two runs each.
set -o pipefail
ALT=${1:-libppfit_prev.so}
B="python -u bench.py --no-legs --cpu-sample 0 --steps 20 --warmup 3"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/ab_new_$i.json 2>/dev/null || exit 1
  PPF_LIB=alt/$ALT timeout -k 10 200 $B > gpurun_out/ab_alt_$i.json 2>/dev/null || exit 1
done
timeout -k 10 150 python -u tools/phase_probe.py > gpurun_out/ph_new.log 2>&1

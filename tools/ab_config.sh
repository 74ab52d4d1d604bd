# A/B of one bench config: the in-tree libppfit.so against alt/$2 (a
# variant build), alternating, two runs each:  tools/ab_config.sh CONFIG LIB
set -o pipefail
CFG=${1:-scattering}
ALT=${2:-libppfit_alt.so}
B="python -u bench.py --config $CFG --no-legs --cpu-sample 0 --steps 10 --warmup 2"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/abc_new_$i.json 2>/dev/null || exit 1
  PPF_LIB=alt/$ALT timeout -k 10 200 $B > gpurun_out/abc_alt_$i.json 2>/dev/null || exit 1
done

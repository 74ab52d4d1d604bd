# bitwise + timing A/B of the working tree's libppfit.so against variants/libppfit_head.so
# usage: ab_scat.sh [quick]
set -e
O=gpurun_out/ab; mkdir -p $O
H=$PWD/pulseportraiture_amd/variants/libppfit_head.so
CASES="headline: headline:exact headline:tnc headline:ncg scattering: scattering:ncg scattering:tnc"
[ "$1" = quick ] && CASES="headline: scattering:"
for c in $CASES; do
  cfg=${c%%:*}; v=${c#*:}; n=1000; [ $cfg = headline ] && n=2000
  PPF_LIB=$H timeout -k 10 200 python3 -u tools/ab_bitwise.py run $O/h_$cfg$v.npz $cfg $n $v
  timeout -k 10 200 python3 -u tools/ab_bitwise.py run $O/n_$cfg$v.npz $cfg $n $v
  python3 tools/ab_bitwise.py cmp $O/h_$cfg$v.npz $O/n_$cfg$v.npz || true
done
PPF_LIB=$H timeout -k 10 240 python3 -u tools/scat_probe.py eval 1000 5
timeout -k 10 240 python3 -u tools/scat_probe.py eval 1000 5
PPF_LIB=$H timeout -k 10 240 python3 -u tools/scat_probe.py fit 1000 3
timeout -k 10 240 python3 -u tools/scat_probe.py fit 1000 3

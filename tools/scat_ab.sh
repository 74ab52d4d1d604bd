# scattering sweep timing per library variant: scat_ab.sh VARIANT... ("base" = in-tree)
set -e
for L in "$@"; do
  if [ $L = base ]; then unset PPF_LIB; else export PPF_LIB=$PWD/pulseportraiture_amd/variants/libppfit_$L.so; fi
  timeout -k 10 240 python3 -u tools/scat_probe.py eval 1000 5 | grep '^{'
  timeout -k 10 240 python3 -u tools/scat_probe.py fit 1000 3 | grep '^{'
done

#!/bin/bash
# Bitwise + timing A/B of library variants on one bench config:
#   tools/ab_variants.sh TAG CONFIG NSUB BASE VARIANT...
# BASE / VARIANT: "tree" (the in-tree libppfit.so) or a name under
# pulseportraiture_amd/variants/ (libppfit_NAME.so).  Per variant: its fit
# outputs against BASE's (tools/ab_bitwise.py cmp), then the bench line of
# every library twice, interleaved.  Each GPU step has its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=$1; C=$2; N=$3; shift 3
O=gpurun_out/$T
mkdir -p $O
lib() { if [ "$1" = tree ]; then unset PPF_LIB; else export PPF_LIB=$R/pulseportraiture_amd/variants/libppfit_$1.so; fi; }
for v in "$@"; do
  lib $v
  timeout -k 10 300 python3 -u tools/ab_bitwise.py run $O/${C}_$v.npz $C $N > $O/bw_${C}_$v.log 2>&1 \
    || { echo "bitwise run $v failed"; tail -5 $O/bw_${C}_$v.log; exit 1; }
done
unset PPF_LIB
B=$1
for v in "${@:2}"; do
  echo "== $C ($N subints): $B vs $v"
  python3 tools/ab_bitwise.py cmp $O/${C}_$B.npz $O/${C}_$v.npz | tail -1
done
for rep in 1 2; do
  for v in "$@"; do
    lib $v
    timeout -k 10 300 python3 -u bench.py --config $C --nsub $N --steps 10 --warmup 2 --cpu-sample 0 --no-legs \
      > $O/bench_${C}_${v}_$rep.json 2> $O/bench_${C}_${v}_$rep.err \
      || { echo "bench $v failed"; tail -5 $O/bench_${C}_${v}_$rep.err; exit 1; }
    python3 - $O/bench_${C}_${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"].get("kernel_ms_per_step", {})
print("%-10s %.3f ms  %s  nfev %.4f" % (sys.argv[2], d["ms_per_step"],
      " ".join("%s %.3f" % (a, b) for a, b in k.items()), d.get("mean_nfev", float("nan"))))
PY
  done
done
unset PPF_LIB
echo AB_VARIANTS_DONE

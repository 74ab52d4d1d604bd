#!/bin/bash
# Timing A/B of library variants on bench configs (no bitwise step):
#   tools/ab_config5.sh TAG "CONFIG[:NSUB] ..." VARIANT...   (VARIANT: tree | variants/ name)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=$1; CFGS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
for cn in $CFGS; do
  c=${cn%%:*}; n=${cn#*:}; [ "$n" = "$cn" ] && n=""
  for rep in 1 2; do
    for v in "$@"; do
      if [ "$v" = tree ]; then unset PPF_LIB; else export PPF_LIB=$R/pulseportraiture_amd/variants/libppfit_$v.so; fi
      timeout -k 10 400 python3 -u bench.py --config $c ${n:+--nsub $n} --steps 5 --warmup 1 --cpu-sample 0 --no-legs \
        > $O/${c}_${v}_$rep.json 2> $O/${c}_${v}_$rep.err || { echo "bench $c $v failed"; tail -5 $O/${c}_${v}_$rep.err; exit 1; }
      python3 - $O/${c}_${v}_$rep.json $c $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"].get("kernel_ms_per_step", {})
print("%-10s %-11s %.3f ms  %s" % (sys.argv[2], sys.argv[3], d["ms_per_step"],
      " ".join("%s %.3f" % (a, b) for a, b in k.items() if b > 0.005)))
PY
    done
  done
done
unset PPF_LIB

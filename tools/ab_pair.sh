#!/bin/bash
# A/B of the in-tree libppfit.so ("new") against a saved variant ("old"):
#   tools/ab_pair.sh TAG OLD CONFIG:NSUB ...
# per config: 1. fit outputs of both libraries (tools/ab_bitwise.py run) and
# their bitwise comparison, 2. the bench line of each (--nsub NSUB, 10 steps),
# alternating old / new / old / new.  Each GPU step has its own time limit;
# the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=$1; OLD=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
OLDLIB=$R/pulseportraiture_amd/variants/libppfit_$OLD.so
for cn in "$@"; do
  c=${cn%%:*}; n=${cn##*:}
  for v in old new; do
    if [ $v = old ]; then export PPF_LIB=$OLDLIB; else unset PPF_LIB; fi
    timeout -k 10 300 python3 -u tools/ab_bitwise.py run $O/${c}_$v.npz $c $n > $O/bw_${c}_$v.log 2>&1 \
      || { echo "bitwise run $c $v failed"; tail -5 $O/bw_${c}_$v.log; exit 1; }
  done
  unset PPF_LIB
  echo "== $c ($n subints): old vs new"
  python3 tools/ab_bitwise.py cmp $O/${c}_old.npz $O/${c}_new.npz
  for rep in 1 2; do
    for v in old new; do
      if [ $v = old ]; then export PPF_LIB=$OLDLIB; else unset PPF_LIB; fi
      timeout -k 10 300 python3 -u bench.py --config $c --nsub $n --steps 10 --warmup 2 --cpu-sample 0 --no-legs \
        > $O/bench_${c}_${v}_$rep.json 2> $O/bench_${c}_${v}_$rep.err \
        || { echo "bench $c $v failed"; tail -5 $O/bench_${c}_${v}_$rep.err; exit 1; }
      python3 - $O/bench_${c}_${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"].get("kernel_ms_per_step", {})
print("%-4s %.3f ms  %s  nfev %.4f" % (sys.argv[2], d["ms_per_step"],
      " ".join("%s %.3f" % (a, b) for a, b in k.items()), d.get("mean_nfev", float("nan"))))
PY
    done
  done
done
unset PPF_LIB
echo AB_PAIR_DONE

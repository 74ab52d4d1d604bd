#!/bin/bash
# Headline bench per library variant: ab_bench.sh TAG VARIANT... ("base" =
# the in-tree libppfit.so; "opt:NAME=V" runs it with a launch-schedule
# option, bench.py --opt NAME=V).  Prints ms/step and the per-kernel HIP-event times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  unset PPF_LIB
  envs=""
  case $v in
    base) ;;
    opt:*) envs="--opt ${v#opt:}" ;;
    *) export PPF_LIB=$R/pulseportraiture_amd/variants/libppfit_$v.so ;;
  esac
  timeout -k 10 300 python3 -u bench.py ${BENCH_ARGS:---steps 5 --warmup 2} $envs --cpu-sample 0 --no-legs > gpurun_out/${T}_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/${T}_$v.log; exit 1; }
  python3 - gpurun_out/${T}_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernel_ms_per_step"]
print("%-14s %.3f ms  %s  nfev %.4f  status %s" % (sys.argv[2], d["ms_per_step"], " ".join("%s %.3f" % (a, b) for a, b in k.items()), d["mean_nfev"], d["status_counts"]))
PY
done

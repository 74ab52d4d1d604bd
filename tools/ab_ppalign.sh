#!/bin/bash
# ppalign (config 5) bench per library variant: ab_ppalign.sh TAG VARIANT...
# ("base" = the in-tree libppfit.so).  Prints ms per iteration and the
# per-iteration kernel times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
T=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  unset PPF_LIB
  [ "$v" = base ] || export PPF_LIB=$R/pulseportraiture_amd/variants/libppfit_$v.so
  timeout -k 10 300 python3 -u bench.py --config ppalign --cpu-sample 0 > gpurun_out/${T}_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/${T}_$v.log; exit 1; }
  python3 - gpurun_out/${T}_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
x = d["detail"]
print("%-8s %.2f ms/iter  calls %s  %s" % (sys.argv[2], x["ms_per_iteration"], x["s_per_call_each"],
      " ".join("%s %.3f" % kv for kv in x["kernel_ms_per_iteration"].items())))
PY
done

#!/bin/bash
# Does the cross-spectrum X stay in the Infinity Cache between the data pass
# and the moment pass?  Per-subint kernel times (HIP events) of the headline
# at growing nsub: X of n subints is n x 1.06 MB.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/xres
mkdir -p $O
for n in 64 128 256 512 1000 4000; do
  timeout -k 10 120 python3 bench.py --nsub $n --steps 10 --warmup 3 --cpu-sample 0 --no-legs > $O/$n.log 2>&1 || { echo "bench $n failed"; tail -3 $O/$n.log; exit 1; }
  python3 - $O/$n.log $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernel_ms_per_step"]
n = int(sys.argv[2])
print(n, "step %.3f ms" % d["ms_per_step"],
      " ".join("%s %.3f us/sub" % (a, 1e3 * k[a] / n) for a in ["data_xspec", "moments", "guess", "fit_taylor", "post"]))
PY
done

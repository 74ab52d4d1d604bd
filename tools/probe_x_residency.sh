#!/bin/bash
# Does the cross-spectrum X stay in the Infinity Cache between the data pass
# and the moment pass?  Per-subint kernel times at growing nsub, non-temporal
# X stores (in-tree library) vs plain stores (libppfit_nt0.so, -DPPF_NT=0).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/xres
mkdir -p $O
python3 - <<'PY' > $O/host.txt
import os
print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())
for p in ["/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"]:
    try:
        print(p, open(p).read().strip())
    except OSError as e:
        print(p, "n/a")
PY
cat $O/host.txt
for lib in default nt0; do
  for n in 100 200 400 1000 4000; do
    if [ $lib = nt0 ]; then export PPF_LIB=$R/pulseportraiture_amd/libppfit_nt0.so; else unset PPF_LIB; fi
    timeout -k 10 120 python3 bench.py --nsub $n --steps 10 --warmup 3 --cpu-sample 0 > $O/${lib}_$n.log 2>&1 || { echo "bench $lib $n failed"; tail -3 $O/${lib}_$n.log; exit 1; }
    python3 - $O/${lib}_$n.log $lib $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernel_ms_per_step"]
n = int(sys.argv[3])
print(sys.argv[2], n, "step %.3f ms" % d["ms_per_step"],
      " ".join("%s %.2f us/sub" % (a, 1e3 * k[a] / n) for a in ["data_xspec", "moments", "guess", "fit_taylor", "post"]))
PY
  done
done

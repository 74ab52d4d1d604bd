#!/bin/bash
# L2 (TCC) hits / misses per kernel of one bench config (one rocprofv3 --pmc
# pass, no trace domains):  tools/pmc_tcc_hits.sh TAG CONFIG NSUB
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; CFG=$2; NF=$3
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
case $CFG in ppalign) P="--nsub $NF --cpu-sample 0";; *) P="--nsub $NF --steps 1 --warmup 0 --cpu-sample 0 --no-timing --no-legs";; esac
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $O/tcc_$CFG -o run --output-format csv -- python3 $R/bench.py --config $CFG $P > $O/tcc_$CFG.log 2>&1 \
  || { echo "pmc failed"; tail -3 $O/tcc_$CFG.log; exit 1; }
python3 - $O/tcc_$CFG <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "TCC_HIT_sum":
        n[k] += 1
for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("TCC_MISS_sum", 0)):
    h, m, rq = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0), v.get("TCC_EA0_RDREQ_sum", 0)
    if h + m < 1e6:
        continue
    print("%-32s launches %3d  hits %.3e  misses %.3e  hit rate %.3f  EA rdreq %.3e  (per launch: misses %.3e)" % (
        k[:32], n[k], h, m, h / max(h + m, 1), rq, m / max(n[k], 1)))
PY

#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 --pmc runs) of one bench
# config with the in-tree library or a variant:
#   tools/pmc_traffic.sh TAG CONFIG NSUB [VARIANT]
# -> gpurun_out/TAG/pmc_traffic_CONFIG[_VARIANT].json (tools/pmc_summary.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; CFG=$2; NF=$3; V=${4:-}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
[ -n "$V" ] && export PPF_LIB=$R/pulseportraiture_amd/variants/libppfit_$V.so
cd /tmp || exit 1
B="$R/bench.py --config $CFG"
S=${V:+_$V}
case $CFG in ppalign) P="--nsub $NF --cpu-sample 0";; *) P="--nsub $NF --steps 1 --warmup 0 --cpu-sample 0 --no-timing --no-legs";; esac
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_${CFG}${S}_$c -o run --output-format csv -- python3 $B $P > $O/pmc_${CFG}${S}_$c.log 2>&1 \
    || { echo "pmc $c failed"; tail -3 $O/pmc_${CFG}${S}_$c.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O/pmc_${CFG}${S}_FETCH_SIZE $O/pmc_${CFG}${S}_WRITE_SIZE $NF $O/pmc_traffic_${CFG}${S}.json "$T $CFG${V:+ ($V)}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, nsub $NF" || exit 1
python3 - $O/pmc_traffic_${CFG}${S}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if v["bytes_per_launch"] > 1e8:
        print("%-28s read %.3f GB write %.3f GB per launch (%d launches)" % (
            k, v["read_bytes_per_launch"] / 1e9, v["write_bytes_per_launch"] / 1e9, v["launches"]))
PY

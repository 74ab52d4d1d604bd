#!/bin/bash
# The round-end checks the driver runs, on one GPU box, each step under its
# own time limit, stopping at the first failure:
#   tools/round_end_check.sh TAG
# 1. pytest -m gpu (verbose, per-test timeout), 2. __graft_entry__.smoke(),
# 3. the default bench line.  Logs under gpurun_out/TAG/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-final}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > $O/gpu_suite.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err \
    || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
echo ROUND_END_CHECK_DONE

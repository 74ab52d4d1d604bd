set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab5
true
true
timeout -k 10 300 python3 -u tools/gettoas_prof_all.py > gpurun_out/ab5/gtprof.log 2>&1 || { echo "gtprof failed"; tail -5 gpurun_out/ab5/gtprof.log; exit 1; }
head -3 gpurun_out/ab5/gtprof.log
timeout -k 10 600 python3 -u bench.py --config gm_shard_host > gpurun_out/ab5/gsh.json 2> gpurun_out/ab5/gsh.err || { echo "gm_shard_host failed"; tail -20 gpurun_out/ab5/gsh.err; exit 1; }
tail -c 1200 gpurun_out/ab5/gsh.json

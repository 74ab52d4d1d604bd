set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab6
timeout -k 10 200 python3 -u tools/prepare_probe.py > gpurun_out/ab6/prep.log 2>&1 || { echo "prep probe failed"; tail -5 gpurun_out/ab6/prep.log; exit 1; }
cat gpurun_out/ab6/prep.log
timeout -k 10 300 python3 -u tools/gettoas_prof_all.py > gpurun_out/ab6/gtprof.log 2>&1 || { echo "gtprof failed"; tail -5 gpurun_out/ab6/gtprof.log; exit 1; }
grep "median ms" gpurun_out/ab6/gtprof.log

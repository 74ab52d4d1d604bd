set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/ab7
timeout -k 10 300 python3 -u tools/gettoas_cprofile.py > gpurun_out/ab7/prep_prof.log 2>&1 || { echo "prep prof failed"; tail -5 gpurun_out/ab7/prep_prof.log; exit 1; }
head -45 gpurun_out/ab7/prep_prof.log

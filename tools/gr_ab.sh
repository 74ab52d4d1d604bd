set -e
mkdir -p gpurun_out/g
BENCH_ARGS="--config scattering --steps 5 --warmup 2" bash tools/ab_bench.sh gr base env:PPF_SCAT_GRAPH=1 base env:PPF_SCAT_GRAPH=1
PPF_SCAT_GRAPH=1 timeout -k 10 200 python3 -u tools/ab_bitwise.py run gpurun_out/g/ng.npz scattering 1000 | grep saved
timeout -k 10 200 python3 -u tools/ab_bitwise.py run gpurun_out/g/g.npz scattering 1000 | grep saved
python3 tools/ab_bitwise.py cmp gpurun_out/g/ng.npz gpurun_out/g/g.npz | tail -1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/g/tests.log 2>&1; tail -2 gpurun_out/g/tests.log
PPF_SCAT_GRAPH=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scattering_floor.py tests/test_gpu_golden_r2.py tests/test_gpu_configs.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/g/tests_graph.log 2>&1; tail -2 gpurun_out/g/tests_graph.log

set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u bench_configs.py --only 1,2,5 --sample 8 > $O/bench_configs.log 2>&1 || { echo "configs failed"; tail -30 $O/bench_configs.log; exit 1; }
cut -c1-300 $O/bench_configs.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -c 3000 $O/bench.log

#!/bin/bash
# Medium / long tier on the GPU box: tests, then the config-3 and medium rows of bench_configs.py
set -o pipefail
TAG=${1:-r03}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_medium.py tests/test_gpu_config3.py tests/test_stitch.py "tests/test_gpu_configs.py::test_config3_annual_5min_window_large_path" "tests/test_gpu_configs.py::test_large_path_with_dcm_columns_in_mixed_batch" -x -v --timeout 180 --timeout-method thread > $O/medium_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/medium_tests.log; exit 1; }
grep -E "PASS|FAIL|config3" $O/medium_tests.log | tail -30
timeout -k 10 600 python -u bench_configs.py --only 3,7 --reps 2 --sample 4 > $O/bench_medium.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_medium.log; exit 1; }
cut -c1-400 $O/bench_medium.log

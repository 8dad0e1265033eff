#!/bin/bash
# Device scenario generator on the GPU box: its tests, the builder / sweep tests, the bench, config 5 end to end
set -o pipefail
TAG=${1:-r03}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_series.py tests/test_gpu_builder.py tests/test_sweep.py -x -v --timeout 300 --timeout-method thread > $O/series_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/series_tests.log; exit 1; }
grep -E "PASS|FAIL" $O/series_tests.log | tail -30
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
python -c "import json,sys; l=json.loads(open('$O/bench.log').read().splitlines()[-1]); print(l['value'], l['ms_per_step'], l['build'], l['end_to_end'], l['roofline']['frac'])"
timeout -k 10 400 python -u bench_configs.py --only 5 --sample 8 > $O/bench_config5.log 2>&1 || { echo "config5 failed"; tail -30 $O/bench_config5.log; exit 1; }
cut -c1-1500 $O/bench_config5.log

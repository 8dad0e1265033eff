#!/bin/bash
# Box form for the ICE windows too: band / config tests, then same-box A/Bs (config 5 and the bench) box on / off.
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_band_scaling.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    echo "== box_$v" >> $O/c5.log
    DVH_BAND_BOX=$v timeout -k 10 300 python -u bench_configs.py --only 5 --c5-scenarios 500 --c5-years 10 >> $O/c5.log 2>&1 || { echo "c5 failed"; tail -20 $O/c5.log; exit 1; }
  done
done
grep -E '^==|^\{' $O/c5.log | cut -c1-330

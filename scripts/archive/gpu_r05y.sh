#!/bin/bash
# New small-window table: GPU tests of the routes, market days at several batch sizes, POI windows by length
set -e
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_market.py tests/test_gpu_cascade.py tests/test_gpu_poi.py > gpurun_out/r05y_tests.log 2>&1
L=gpurun_out/r05y_market_table2.log
: > $L
timeout -k 10 240 python -u scripts/probe_market_variants.py >> $L 2>&1
for d in 5 40 122; do
  MARKET_DAYS=$d timeout -k 10 240 python -u scripts/probe_market_variants.py fr,reserves,lf,lf_combined >> $L 2>&1
done
timeout -k 10 300 python -u scripts/probe_poi_paths.py 64 > gpurun_out/r05y_poi_paths2.log 2>&1

#!/bin/bash
# Objective gate with the dual-residual term (band forms): band tests, certification dump, bench.
set -o pipefail
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_band_scaling.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/certify_dump.py --label r04y --blend 4 > $O/certify.log 2>&1 || { echo "dump failed"; tail -20 $O/certify.log; exit 1; }
grep -E "seeded|cold" $O/certify.log
timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-250

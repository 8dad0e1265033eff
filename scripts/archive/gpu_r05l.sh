#!/bin/bash
# Cost prefetch across the barrier (kCostPrefetch) vs without: fixed-iteration speed; band tests.
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue_cpre.log 2>&1 || { echo "cpre failed"; tail -20 $O/queue_cpre.log; exit 1; }
DVH_LIB=scripts/_variants/lib_nocpre.so timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue_nocpre.log 2>&1 || { echo "nocpre failed"; tail -20 $O/queue_nocpre.log; exit 1; }
grep -H queue $O/queue_*.log | cut -c1-150
timeout -k 10 400 python -u -m pytest tests/test_gpu_band_scaling.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log

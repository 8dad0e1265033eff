#!/bin/bash
# Tau column updated in the dual half-step (kTauDual): fixed-iteration speed vs the wave-0 form, anatomy, band tests.
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 200 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue.log 2>&1 || { echo "queue probe failed"; tail -20 $O/queue.log; exit 1; }
DVH_LIB=scripts/_variants/lib_tau0.so timeout -k 10 200 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue_tau0.log 2>&1 || { echo "queue tau0 probe failed"; tail -20 $O/queue_tau0.log; exit 1; }
grep queue $O/queue.log $O/queue_tau0.log
DVH_LIB=scripts/_variants/lib_probe.so timeout -k 10 200 python -u scripts/probe_band_latency.py 5000 1024 > $O/latency.log 2>&1 || { echo "latency probe failed"; tail -20 $O/latency.log; exit 1; }
grep -v amdgpu.ids $O/latency.log | grep -v "^  wave\|SIMD"
timeout -k 10 400 python -u -m pytest tests/test_gpu_band_scaling.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log

#!/bin/bash
# The persistent-vs-one-workgroup parity tests (battery, ICE).
set -o pipefail
O=gpurun_out/r04ap; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_band_scaling.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -12

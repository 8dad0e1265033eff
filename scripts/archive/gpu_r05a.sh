#!/bin/bash
# Round 5 first pass: drop-in relaxation / retry, cascade -2 re-route, per-handle slot cache -- full GPU suite + bench.
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300

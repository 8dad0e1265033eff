#!/bin/bash
# Objective gate with the dual-residual term in every kernel and both restatements: full GPU suite, certification,
# bench, configs 1/2/3/5.
set -o pipefail
O=gpurun_out/r04z; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u scripts/certify_dump.py --label r04z --blend 4 > $O/certify.log 2>&1 || { echo "dump failed"; tail -20 $O/certify.log; exit 1; }
grep -E "seeded|cold" $O/certify.log | cut -c1-80
timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
timeout -k 10 700 python -u bench_configs.py --only 1,2,3,5 --sample 16 > $O/bench_configs.log 2>&1 || { echo "configs failed"; tail -30 $O/bench_configs.log; exit 1; }
grep '^{' $O/bench_configs.log | cut -c1-150

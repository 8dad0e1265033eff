#!/bin/bash
# Round-4 pass on the persistent band form: full GPU suite, smoke, bench (driver form), configs.
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300
timeout -k 10 600 python -u bench_configs.py --only 1,2,5 --sample 16 > $O/bench_configs.log 2>&1 || { echo "configs failed"; tail -30 $O/bench_configs.log; exit 1; }
grep '^{' $O/bench_configs.log | cut -c1-200

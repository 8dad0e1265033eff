#!/bin/bash
# Validation: full GPU suite, smoke, config 5 (ICE form back on the round-3 gate), bench.
set -o pipefail
O=gpurun_out/r04ac; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-120
timeout -k 10 300 python -u bench_configs.py --only 5 > $O/c5.log 2>&1 || { echo "c5 failed"; tail -20 $O/c5.log; exit 1; }
grep '^{' $O/c5.log | python -c "import json,sys; [print(json.loads(l)['windows_per_s'], json.loads(l)['solve_ms_total']) for l in sys.stdin]"
timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-160

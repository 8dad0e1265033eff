#!/bin/bash
# Last check of the committed tree: GPU suite, smoke, and bench.py with no flags (the driver's default invocation)
set -o pipefail
O=gpurun_out/r05zv; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-150
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['steps'], d['roofline']['frac'], d['cpu_baseline']['value'])"

#!/bin/bash
# Full GPU suite + smoke on the current sources, then the full-population certification dump (seeded + cold).
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
timeout -k 10 400 python -u scripts/certify_dump.py --label r05t --blend 4 > $O/certify.log 2>&1 || { echo "dump failed"; tail -20 $O/certify.log; exit 1; }
grep -E "seeded|cold" $O/certify.log | cut -c1-120

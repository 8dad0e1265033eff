#!/bin/bash
# Last validation of the round: full GPU suite (with the market-options test), then the 2-rank rehearsal.
set -o pipefail
O=gpurun_out/r04ai; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash scripts/rehearse_2rank.sh r04ai_rehearse 2000 || exit 1

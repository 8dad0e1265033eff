#!/bin/bash
# Box steps rescaled at restarts and width-free movement norms (kBoxRescale) vs the width re-reads: check schedules
# at a fixed iteration count; band / sweep GPU tests; a short bench.
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 200 python -u scripts/probe_check_cost.py 5000 1024 > $O/cost_rstep1.log 2>&1 || { echo "rstep1 failed"; tail -20 $O/cost_rstep1.log; exit 1; }
DVH_LIB=scripts/_variants/lib_rstep0.so timeout -k 10 200 python -u scripts/probe_check_cost.py 5000 1024 > $O/cost_rstep0.log 2>&1 || { echo "rstep0 failed"; tail -20 $O/cost_rstep0.log; exit 1; }
paste <(grep check_every $O/cost_rstep0.log | cut -c1-100) <(grep check_every $O/cost_rstep1.log | cut -c60-100)
timeout -k 10 400 python -u -m pytest tests/test_gpu_band_scaling.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
DVH_LIB=scripts/_variants/lib_rstep0.so timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 > $O/bench0.log 2>&1 || { echo "bench0 failed"; tail -20 $O/bench0.log; exit 1; }
grep '^{' $O/bench0.log | cut -c1-200

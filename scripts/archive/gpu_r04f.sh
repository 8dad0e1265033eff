#!/bin/bash
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
DVH_CHAIN_PROBE_DUMP=1 DVH_LIB=scripts/_variants/lib_ctime3.so timeout -k 10 240 python -u scripts/probe_chain.py --iters 8192 da dcm_nopv dcm year64 > $O/probe_chain.log 2>&1 || { echo "probe failed"; tail -20 $O/probe_chain.log; exit 1; }
for v in da dcm_nopv dcm; do
  timeout -k 10 120 python -u scripts/prof_config3.py $v >> $O/config3.log 2>&1 || { echo "config3 $v failed"; tail -20 $O/config3.log; exit 1; }
done
grep '^{' $O/config3.log | cut -c1-150
timeout -k 10 400 python -u -m pytest tests/test_gpu_medium.py tests/test_gpu_config3.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u bench_configs.py --only 7 > $O/medium.log 2>&1 || { echo "medium failed"; tail -30 $O/medium.log; exit 1; }
grep '^{' $O/medium.log | cut -c1-300

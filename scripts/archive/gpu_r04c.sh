#!/bin/bash
# Team kernel: the tau exchange waited in the dual half-step (default) vs the primal half-step (round 3), fixed-iteration
# probe and converged config-3 solves; then the medium / config-3 GPU tests on the default build.
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
for r in 1 2; do
for v in ctauD ctauP; do
  echo "== $v" >> $O/probe_chain.log
  DVH_LIB=scripts/_variants/lib_$v.so timeout -k 10 240 python -u scripts/probe_chain.py --iters 8192 da dcm_nopv dcm year64 >> $O/probe_chain.log 2>&1 || { echo "$v failed"; tail -20 $O/probe_chain.log; exit 1; }
done
done
for v in da dcm_nopv dcm; do
  timeout -k 10 120 python -u scripts/prof_config3.py $v >> $O/config3.log 2>&1 || { echo "config3 $v failed"; tail -20 $O/config3.log; exit 1; }
done
grep '^{' $O/config3.log | cut -c1-220
timeout -k 10 400 python -u -m pytest tests/test_gpu_medium.py tests/test_gpu_config3.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log

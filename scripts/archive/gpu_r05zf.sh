#!/bin/bash
# Warm transfer with the partners' offsets hoisted and each chunk's loads issued first: bench A/B against the HEAD
# library (ab_libs/lib_head.so) -- the warm_transfer_kernel time and the iteration statistics must match exactly
set -o pipefail
O=gpurun_out/r05zf; mkdir -p $O
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sweep.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for L in head cur head cur; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_$L.log 2>&1 || { echo "$L failed"; tail -20 $O/bench_$L.log; exit 1; }
  echo $L $(tail -1 $O/bench_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'], d['kernel_ms'])")
done

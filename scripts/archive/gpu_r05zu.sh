#!/bin/bash
# Persistent band units with the write-back re-derived (DVH_BAND_REDERIVE): band GPU tests, then bench and config 5
# against the HEAD library (ab_libs/lib_head.so), alternating, same box
set -o pipefail
O=gpurun_out/r05zu; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band_scaling.py tests/test_gpu_configs.py tests/test_sweep.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for L in head cur head cur; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_$L.log 2>&1 || { echo "$L bench failed"; tail -20 $O/bench_$L.log; exit 1; }
  timeout -k 10 300 python -u bench_configs.py --only 5 --sample 0 > $O/c5_$L.log 2>&1 || { echo "$L c5 failed"; tail -20 $O/c5_$L.log; exit 1; }
  echo $L bench $(tail -1 $O/bench_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'])") c5 $(grep '"config5"' $O/c5_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d['iters_mean'])")
done

#!/bin/bash
# KKT helpers out of line in the ICE form only: config 5 vs the 064ed27 library (helpers out of line everywhere), bench
set -o pipefail
O=gpurun_out/r05zb; mkdir -p $O
for L in 064ed27 cur; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench_configs.py --only 5 --sample 0 > $O/c5_$L.log 2>&1 || { echo "$L failed"; tail -20 $O/c5_$L.log; exit 1; }
  echo $L $(grep '"config5"' $O/c5_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d['iters_mean'])")
done
unset DVH_LIB
timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200

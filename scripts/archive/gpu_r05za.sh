#!/bin/bash
# Config 5 bisection over round-5 libraries (ab_libs/lib_<commit>.so, built from those commits) vs the current one
set -o pipefail
O=gpurun_out/r05za; mkdir -p $O
for L in r04 69d390d a617129 064ed27 b9afaf5 cur; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench_configs.py --only 5 --sample 0 > $O/bis_$L.log 2>&1 || { echo "$L failed"; tail -20 $O/bis_$L.log; exit 1; }
  echo $L $(grep '"config5"' $O/bis_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d['iters_mean'])")
done

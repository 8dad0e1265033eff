#!/bin/bash
# ICE persistent unit with further scheduler options (ab_libs/lib_<v>.so): config 5, same box
set -o pipefail
O=gpurun_out/r05zm; mkdir -p $O
for L in cur i_nocluster i_relaxocc i_itilp i_nopostrasink cur; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench_configs.py --only 5 --sample 0 > $O/c5_$L.log 2>&1 || { echo "$L failed"; tail -20 $O/c5_$L.log; exit 1; }
  echo $L c5 $(grep '"config5"' $O/c5_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d['iters_mean'])")
done

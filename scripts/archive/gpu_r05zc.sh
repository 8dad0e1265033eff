#!/bin/bash
# Config 5: ICE box form (DVH_BAND_BOX=2) vs default, twice each, same box
set -o pipefail
O=gpurun_out/r05zc; mkdir -p $O
for i in 1 2; do
for V in def box2; do
  if [ $V = box2 ]; then export DVH_BAND_BOX=2; else unset DVH_BAND_BOX; fi
  timeout -k 10 300 python -u bench_configs.py --only 5 --sample 16 > $O/c5_${V}_$i.log 2>&1 || { echo "$V failed"; tail -20 $O/c5_${V}_$i.log; exit 1; }
  echo $V $(grep '"config5"' $O/c5_${V}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d['iters_mean'], d['optimal'], d['parity_year0']['max_obj_rel_err_vs_highs'])")
done
done

#!/bin/bash
# Blend weights moved toward the partners' affine combination reproducing the window's features (bench.py --blend-lam),
# against inverse-distance weights, bench, same box
set -o pipefail
O=gpurun_out/r05zx; mkdir -p $O
for cfg in "4 -1" "8 1" "4 1" "6 1" "8 3" "8 0.3" "4 -1"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 6 --warmup 2 --blend $1 --blend-lam $2 > $O/b_$1_$2.log 2>&1 || { echo "$cfg failed"; tail -20 $O/b_$1_$2.log; exit 1; }
  echo "blend $1 lam $2" $(tail -1 $O/b_$1_$2.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); s=d['schedule']; print(d['value'], d['ms_per_step'], d['iters_mean'], s['iters_mean_warm'], d['max_primal_res_rel'], d['optimal_frac'])")
done

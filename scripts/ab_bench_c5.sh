#!/bin/bash
# A/B of library builds on the bench (bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3, alternating, 3 rounds) and
# on config 5 (bench_configs.py --only 5 --sample 0, 2 rounds).  Usage: scripts/ab_bench_c5.sh <outdir> <lib> <lib> ...
# (ab_libs/lib_<name>.so); prints value, ms/step, iters mean, max primal residual / windows/s, solve ms
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2 3; do
  for L in "$@"; do
    export DVH_LIB=ab_libs/lib_$L.so
    timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_${L}_$r.log 2>&1 || { echo "$L bench failed"; tail -20 $O/bench_${L}_$r.log; exit 1; }
    echo $L bench $(tail -1 $O/bench_${L}_$r.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'])")
  done
done
for r in 1 2; do
  for L in "$@"; do
    export DVH_LIB=ab_libs/lib_$L.so
    timeout -k 10 400 python -u bench_configs.py --only 5 --sample 0 > $O/c5_${L}_$r.log 2>&1 || { echo "$L c5 failed"; tail -20 $O/c5_${L}_$r.log; exit 1; }
    echo "$L c5 $(grep '"config5"' $O/c5_${L}_$r.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d['iters_mean'])")"
  done
done

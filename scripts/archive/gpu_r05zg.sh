#!/bin/bash
# AMDGPU scheduler options on the persistent band translation unit (ab_libs/lib_<v>.so from dervet_hip.build.build_variant):
# config 5 (ICE form) and the bench (battery form) against the default build, same box
set -o pipefail
O=gpurun_out/r05zg; mkdir -p $O
for L in cur maxilp minreg bias100 trackers nounclust cur; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench_configs.py --only 5 --sample 0 > $O/c5_$L.log 2>&1 || { echo "$L c5 failed"; tail -20 $O/c5_$L.log; exit 1; }
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 6 --warmup 2 > $O/bench_$L.log 2>&1 || { echo "$L bench failed"; tail -20 $O/bench_$L.log; exit 1; }
  echo $L c5 $(grep '"config5"' $O/c5_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d['iters_mean'])") bench $(tail -1 $O/bench_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'])")
done

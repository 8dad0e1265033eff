#!/bin/bash
# wave 0's Halpern blends pinned before the second barrier (DVH_BAND_PIN_BLEND), A/B on the bench and the fixed-iteration probe
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
for L in cur pin cur pin cur pin; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_$L.log 2>&1 || { echo "$L bench failed"; tail -20 $O/bench_$L.log; exit 1; }
  echo $L bench $(tail -1 $O/bench_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'])")
done
for L in cur pin; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/probe_$L.log 2>&1 || { echo "$L probe failed"; exit 1; }
  echo "$L $(tail -1 $O/probe_$L.log)"
done

#!/bin/bash
# own-column K x-bar pinned before the first barrier on waves 1-3 (DVH_BAND_PIN_KX), A/B on the bench, probe and config 5
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
for L in base pinkx base pinkx base pinkx; do
  export DVH_LIB=ab_libs/lib_$L.so
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_$L.log 2>&1 || { echo "$L bench failed"; tail -20 $O/bench_$L.log; exit 1; }
  echo $L bench $(tail -1 $O/bench_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'])")
done
for L in base pinkx; do
  export DVH_LIB=ab_libs/lib_$L.so
  timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/probe_$L.log 2>&1 || { echo "$L probe failed"; exit 1; }
  echo "$L $(tail -1 $O/probe_$L.log)"
  timeout -k 10 400 python -u bench_configs.py --only 5 --sample 0 > $O/c5_$L.log 2>&1 || { echo "$L c5 failed"; exit 1; }
  echo "$L c5 $(grep '"config5"' $O/c5_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'])")"
done

#!/bin/bash
# lane-local SOE rows after the second barrier (DVH_BAND_LATE_SOE) on top of the pinned blends; config 5 / 1 / 2 with and
# without the pinned blends
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
for L in cur late cur late; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_$L.log 2>&1 || { echo "$L bench failed"; tail -20 $O/bench_$L.log; exit 1; }
  echo $L bench $(tail -1 $O/bench_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'])")
done
for L in cur pin0 late; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 400 python -u bench_configs.py --only 1,2,5 --sample 0 > $O/configs_$L.log 2>&1 || { echo "$L configs failed"; tail -20 $O/configs_$L.log; exit 1; }
  echo "$L configs"; grep -h '"config' $O/configs_$L.log | python -c "
import sys, json
for l in sys.stdin:
    try: d = json.loads(l)
    except Exception: continue
    print('  ', d.get('config'), d.get('windows_per_s'), d.get('solve_ms_total', d.get('ms')), d.get('iters_mean'))"
done

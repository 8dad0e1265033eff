#!/bin/bash
# Round 6: the full GPU suite on the new default library (wave-0 priority on), then bench steps of the priority
# variants and configs 1 / 2 / 5 against the round-5 library and the ICE form without the batched factor loads.
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for L in cur prio3 pdual prio0 cur prio3 pdual prio0; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_$L.log 2>&1 || { echo "$L bench failed"; tail -20 $O/bench_$L.log; exit 1; }
  echo $L bench $(tail -1 $O/bench_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'])")
done
for L in cur prio0 pfice0 r5; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 400 python -u bench_configs.py --only 1,2,5 --sample 0 > $O/configs_$L.log 2>&1 || { echo "$L configs failed"; tail -20 $O/configs_$L.log; exit 1; }
  echo "$L configs"; grep -h '"config' $O/configs_$L.log | python -c "
import sys, json
for l in sys.stdin:
    try: d = json.loads(l)
    except Exception: continue
    print('  ', d.get('config'), d.get('windows_per_s'), d.get('solve_ms_total', d.get('ms')), d.get('iters_mean'))"
done
echo all done

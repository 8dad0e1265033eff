#!/bin/bash
# (1) bit-identity of the round-6 band kernel with round 5's on the bench batch (SHA-256 of x, y, stats, istats after a
# seeded step), (2) the chain kernel's batched KKT factor loads and hand-off wave priority on config 3 and the medium
# tier, against round 5
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
for L in cur r5; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 3 --warmup 1 --sha > $O/sha_$L.log 2>&1 || { echo "$L sha failed"; tail -20 $O/sha_$L.log; exit 1; }
  echo $L $(tail -1 $O/sha_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['iters_mean'], d['outputs_sha256'])")
done
unset DVH_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_config3.py tests/test_gpu_medium.py > $O/chain_tests.log 2>&1 || { echo "chain tests failed"; tail -30 $O/chain_tests.log; exit 1; }
tail -1 $O/chain_tests.log
for L in cur chainpf0 chainprio r5; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 500 python -u bench_configs.py --only 3,7 --sample 0 --reps 2 > $O/c37_$L.log 2>&1 || { echo "$L configs failed"; tail -20 $O/c37_$L.log; exit 1; }
  echo "$L"; grep -h '"config' $O/c37_$L.log | python -c "
import sys, json
for l in sys.stdin:
    try: d = json.loads(l)
    except Exception: continue
    print('  ', d.get('config'), d.get('note', '')[:40], d.get('windows_per_s'), d.get('solve_ms_total', d.get('ms')), d.get('iters_mean'))"
done
echo all done

#!/bin/bash
# Round 6, first pass: GPU tests of the drop-in / band paths on the new library (single-precision-exact factors, no
# width round trip, Halpern weights divided in the lanes), then per-iteration probes and bench steps against the
# round-5 library and the A/B variants (wave-0 priority, early SOE rows), alternating, same box.
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_export.py tests/test_gpu_band_scaling.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_benefit.py tests/test_sweep.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for L in r5 cur pf0 early prio ep; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/probe_$L.log 2>&1 || { echo "$L probe failed"; tail -20 $O/probe_$L.log; exit 1; }
  echo "$L $(tail -1 $O/probe_$L.log)"
done
for L in r5 cur pf0 early prio ep r5 cur pf0 early prio ep; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_$L.log 2>&1 || { echo "$L bench failed"; tail -20 $O/bench_$L.log; exit 1; }
  echo $L bench $(tail -1 $O/bench_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'])")
done
echo all done

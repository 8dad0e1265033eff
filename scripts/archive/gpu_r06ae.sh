#!/bin/bash
# chain kernel: local tau update in the primal half-step with the tau wave at raised priority (DVH_CHAIN_TAU_LOCAL=2), A/B
# and the medium tier (bench_configs.py --only 3,7 --sample 0) and the fixed-iteration probe; then the medium / config-3
# GPU tests on the new default build
set -o pipefail
O=gpurun_out/r06ae; mkdir -p $O
for r in 1 2; do
  for L in cbase tlp; do
    export DVH_LIB=ab_libs/lib_$L.so
    timeout -k 10 400 python -u bench_configs.py --only 3,7 --sample 0 > $O/cfg_${L}_$r.log 2>&1 || { echo "$L configs failed"; tail -20 $O/cfg_${L}_$r.log; exit 1; }
    echo "$L $(grep '^{' $O/cfg_${L}_$r.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'], d.get('schedule'), d.get('wall_ms'), d.get('windows_per_s'), end=' | ')")"
  done
done
for L in cbase tlp; do
  export DVH_LIB=ab_libs/lib_$L.so
  timeout -k 10 300 python -u scripts/probe_chain.py --iters 8192 dcm year64 > $O/probe_$L.log 2>&1 || { echo "$L probe failed"; tail -20 $O/probe_$L.log; exit 1; }
  echo "== probe $L"; grep '^{' $O/probe_$L.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['variant'], d['windows'], d['iters'], d['pdhg_ms'], d['us_per_iter'])"
done
unset DVH_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_medium.py tests/test_gpu_config3.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log

#!/bin/bash
# Chain and ELL / generic units built without machine LICM: their GPU tests, configs 3 / market / medium, POI windows
set -o pipefail
O=gpurun_out/r05zk; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_medium.py tests/test_gpu_config3.py tests/test_gpu_market.py tests/test_gpu_poi.py tests/test_gpu_cascade.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u bench_configs.py --only 3,6,7 > $O/cfg.log 2>&1 || { echo "cfg failed"; tail -20 $O/cfg.log; exit 1; }
grep '^{' $O/cfg.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config'], d.get('schedule'), d.get('wall_ms'), d.get('windows_per_s'), d.get('iters_mean'), (d.get('parity') or {}).get('max_obj_rel_err_vs_highs'))"
timeout -k 10 300 python -u scripts/probe_poi_paths.py 64 month > $O/poi.log 2>&1 || { echo "poi failed"; tail -20 $O/poi.log; exit 1; }
grep -v amdgpu $O/poi.log | cut -c1-200

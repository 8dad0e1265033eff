#!/bin/bash
# Market-service days with scenarios.MARKET_OPTIONS (theta 0.5): market tests, market configs.
set -o pipefail
O=gpurun_out/r04ag; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_market.py tests/test_gpu_cascade.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench_configs.py --only 6 --sample 16 > $O/market.log 2>&1 || { echo "market failed"; tail -20 $O/market.log; exit 1; }
grep '^{' $O/market.log | python -c "
import json,sys
for l in sys.stdin:
    j=json.loads(l); print(j['config'], j['wall_ms'], j['windows_per_s'], j['iters_mean'], j['iters_max'], (j.get('parity') or {}).get('max_obj_rel_err_vs_highs'), j.get('options'))"

#!/bin/bash
# The ICE pass in the caller's launch order (route over the order): config 5 with / without the warm order, GPU suite,
# PMC passes of the bench (new source key), bench.
set -o pipefail
O=gpurun_out/r04ar; mkdir -p $O
for r in 1 2; do
  for v in 1 0; do
    echo "== order_$v" >> $O/c5.log
    DVH_SWEEP_ORDER=$v timeout -k 10 300 python -u bench_configs.py --only 5 --sample 16 >> $O/c5.log 2>&1 || { echo "config5 failed"; tail -20 $O/c5.log; exit 1; }
  done
done
python3 -c "
import json
cur=None
for l in open('$O/c5.log'):
    if l.startswith('=='): cur=l.strip()
    elif l.startswith('{'):
        d=json.loads(l); print(cur, 'config5 windows/s', d.get('windows_per_s'), 'iters', d.get('iters_mean'), 'obj err vs HiGHS', d['parity_year0']['max_obj_rel_err_vs_highs'])
"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
scripts/profile_round.sh r04ar || exit 1
cp gpurun_out/prof_r04ar/pdhg_valu.json gpurun_out/prof_r04ar/pdhg_traffic.json profiles/ || exit 1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300

#!/bin/bash
# With the persistent forms built without machine LICM: does the warm launch order still pay (DVH_SWEEP_ORDER=0 vs the
# seed predictor), and does the ICE box form (DVH_BAND_BOX=2) pay on config 5 now?
set -o pipefail
O=gpurun_out/r04aq; mkdir -p $O
for r in 1 2; do
  for v in 1 0; do
    echo "== order_$v" >> $O/ab.log
    DVH_SWEEP_ORDER=$v timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
  done
done
python scripts/ab_summary.py $O/ab.log
for r in 1 2; do
  for b in 1 2; do
    echo "== ice_box_$b" >> $O/c5.log
    DVH_BAND_BOX=$b timeout -k 10 300 python -u bench_configs.py --only 5 --sample 16 >> $O/c5.log 2>&1 || { echo "config5 failed"; tail -20 $O/c5.log; exit 1; }
  done
done
python3 -c "
import json
cur=None
for l in open('$O/c5.log'):
    if l.startswith('=='): cur=l.strip()
    elif l.startswith('{'):
        d=json.loads(l); print(cur, d.get('windows_per_s'), d.get('iters_mean'), d['parity_year0']['max_obj_rel_err_vs_highs'])
"

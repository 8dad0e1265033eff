#!/bin/bash
# A/B: the ICE band form persistent (DVH_BAND_QUEUE_ICE=1, built in dvh_band_persist.hip without machine LICM) vs one
# workgroup per window, on config 5.
set -o pipefail
O=gpurun_out/r04an; mkdir -p $O
for r in 1 2; do
  for q in 0 1; do
    echo "== ice_queue_$q" >> $O/ab.log
    DVH_BAND_QUEUE_ICE=$q timeout -k 10 300 python -u bench_configs.py --only 5 --sample 16 >> $O/ab.log 2>&1 || { echo "config5 failed"; tail -20 $O/ab.log; exit 1; }
  done
done
grep "^==\|config5" $O/ab.log | cut -c1-330

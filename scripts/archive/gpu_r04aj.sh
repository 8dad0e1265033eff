#!/bin/bash
# Where the persistent form stands against the sorted ceiling: {persistent, one workgroup per window} x {seed-predictor
# order, the previous step's own counts (diagnostic ceiling)}.
set -o pipefail
O=gpurun_out/r04aj; mkdir -p $O
for r in 1 2; do
  for q in 1 0; do
    for v in 1 prev; do
      echo "== q${q}_order_${v}" >> $O/ab.log
      DVH_BAND_QUEUE=$q DVH_SWEEP_ORDER=$v timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
    done
  done
done
python scripts/ab_summary.py $O/ab.log

#!/bin/bash
# Launch-order ceiling: packing order vs the previous step's own iteration counts (perfect LPT) vs the seed predictor.
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
for r in 1 2; do
  for v in 0 prev 1; do
    echo "== order_$v" >> $O/ab.log
    DVH_SWEEP_ORDER=$v timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
  done
done
python scripts/ab_summary.py $O/ab.log

#!/bin/bash
# Launch-order study (band pass of the warm phase): packing, random, previous counts descending / ascending.
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
for r in 1 2; do
  for v in 0 random prev prevasc; do
    echo "== order_$v" >> $O/ab.log
    DVH_SWEEP_ORDER=$v timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
  done
done
python scripts/ab_summary.py $O/ab.log

#!/bin/bash
# Power-iteration steps for ||K~||_2 (dvh_options.power_iters, default 64) on the bench workload: seeded and cold time,
# iterations (certify_dump: every window's objective for scripts/certify_highs.py)
set -o pipefail
O=gpurun_out/r05zn; mkdir -p $O
for P in 64 24 16 12 8; do
  timeout -k 10 300 python -u scripts/certify_dump.py --label pw$P --blend 4 --opt power_iters=$P > $O/pw$P.log 2>&1 || { echo "$P failed"; tail -20 $O/pw$P.log; exit 1; }
  echo power_iters=$P $(grep -E "seeded|cold" $O/pw$P.log | cut -c1-60)
done

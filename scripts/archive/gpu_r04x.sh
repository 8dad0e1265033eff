#!/bin/bash
# Certification at tighter KKT tolerances (seeded): eps 9e-7 and 8e-7.
set -o pipefail
O=gpurun_out/r04x; mkdir -p $O
for e in 9e-7 8e-7; do
  timeout -k 10 300 python -u scripts/certify_dump.py --label r04x_eps$e --blend 4 --no-cold --eps $e >> $O/certify.log 2>&1 || { echo "dump failed"; tail -20 $O/certify.log; exit 1; }
done
grep -E "seeded|wrote" $O/certify.log

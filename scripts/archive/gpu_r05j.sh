#!/bin/bash
# Overlap in bench.py's order (gather enqueued before the next solve) at 2 and 15 GiB, no reservation.
set -o pipefail
O=gpurun_out/r05j; mkdir -p $O
for g in 2 15; do
  timeout -k 10 200 python -u scripts/probe_overlap.py 4000 $g > $O/overlap_g$g.log 2>&1 || { echo "overlap g$g failed"; tail -20 $O/overlap_g$g.log; exit 1; }
  grep -v amdgpu.ids $O/overlap_g$g.log
done

#!/bin/bash
# Per-iteration speed of the persistent vs one-workgroup band forms at equal window durations.
set -o pipefail
O=gpurun_out/r04ak; mkdir -p $O
for r in 1 2; do
  for q in 1 0; do
    DVH_BAND_QUEUE=$q timeout -k 10 300 python -u scripts/probe_band_queue.py 5000 1024 >> $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
  done
done
grep queue= $O/probe.log

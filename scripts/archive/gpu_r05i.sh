#!/bin/bash
# Overlap of a 2 GiB copy (RCCL all-gather stand-in) with the persistent band grid, with 0 / 8 / 32 CUs' slots reserved.
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
for r in 0 8 32; do
  DVH_BAND_RESERVE=$r timeout -k 10 200 python -u scripts/probe_overlap.py 4000 2 > $O/overlap_r$r.log 2>&1 || { echo "overlap r$r failed"; tail -20 $O/overlap_r$r.log; exit 1; }
  grep -v amdgpu.ids $O/overlap_r$r.log
done

#!/bin/bash
# Market-day routing A/B over the small ELL variants (scripts/probe_market_variants.py)
set -e
L=gpurun_out/r05w_market_variants.log
: > $L
timeout -k 10 240 python -u scripts/probe_market_variants.py >> $L 2>&1
for v in -1 0 1 2 3 4 5 6; do
  DVH_SMALL=$v timeout -k 10 240 python -u scripts/probe_market_variants.py >> $L 2>&1
done

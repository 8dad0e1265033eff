#!/bin/bash
# Small ELL variant candidates for market days (scripts/probe_market_variants.py; the candidates were temporary
# DVH_SMALL cases 7-23 in dvh_kernels.hip small_dispatch: profiles/r05x_market_candidates*.log name them by variant code)
set -e
L=gpurun_out/r05x_market_candidates2.log
: > $L
for v in 12 13 14 15 16 17 18 19; do
  DVH_SMALL=$v timeout -k 10 240 python -u scripts/probe_market_variants.py >> $L 2>&1
done

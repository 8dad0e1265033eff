#!/bin/bash
# Ablation upper bounds (wrong results, timing only): no cost/rhs LDS reads (8), no neighbour LDS reads (16), both (24),
# everything (31: + no barriers + no tau chain).
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue_base.log 2>&1 || { echo "base failed"; tail -20 $O/queue_base.log; exit 1; }
for v in abl8 abl16 abl24 abl3 abl31; do
  DVH_LIB=scripts/_variants/lib_$v.so timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue_$v.log 2>&1 || { echo "$v failed"; tail -20 $O/queue_$v.log; exit 1; }
done
grep -H queue $O/queue_*.log | cut -c1-150

#!/bin/bash
# Ablation upper bounds (wrong results, timing only) at a fixed iteration count: no barrier 1 / 2 / both, no tau chain.
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue_base.log 2>&1 || { echo "base failed"; tail -20 $O/queue_base.log; exit 1; }
for v in abl1 abl2 abl3 abl4 abl5 taud; do
  DVH_LIB=scripts/_variants/lib_$v.so timeout -k 10 120 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue_$v.log 2>&1 || { echo "$v failed"; tail -20 $O/queue_$v.log; exit 1; }
done
grep -H queue $O/queue_*.log

#!/bin/bash
# Per-wave tau sums (DVH_BAND_TAU_WAVESUMS=1) vs wave 0's reduction, battery (config 4) and ICE (config 5) forms,
# fixed iteration count.
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
for c in config4 config5; do
  S=5000; [ $c = config5 ] && S=1000
  timeout -k 10 120 python -u scripts/probe_band_queue.py $S 1024 $c > $O/base_$c.log 2>&1 || { echo "base $c failed"; tail -20 $O/base_$c.log; exit 1; }
  DVH_LIB=scripts/_variants/lib_tws.so timeout -k 10 120 python -u scripts/probe_band_queue.py $S 1024 $c > $O/tws_$c.log 2>&1 || { echo "tws $c failed"; tail -20 $O/tws_$c.log; exit 1; }
done
grep -H queue $O/*.log | cut -c1-150

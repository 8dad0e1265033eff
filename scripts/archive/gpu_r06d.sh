#!/bin/bash
# Where a band iteration goes with wave 0 at raised priority (per-wave shader-clock probe, fixed 1,024 iterations), and
# what a check costs now (fixed iterations under different check schedules), against the round-5 library
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
for L in probe probe_p0; do
  DVH_LIB=ab_libs/lib_$L.so timeout -k 10 180 python -u scripts/probe_band_latency.py 2000 1024 > $O/lat_$L.log 2>&1 || { echo "$L latency failed"; tail -20 $O/lat_$L.log; exit 1; }
  echo "== $L"; tail -5 $O/lat_$L.log
done
for L in cur r5; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 400 python -u scripts/probe_check_cost.py 5000 1024 > $O/checks_$L.log 2>&1 || { echo "$L checks failed"; tail -20 $O/checks_$L.log; exit 1; }
  echo "== $L"; cat $O/checks_$L.log
done
echo all done

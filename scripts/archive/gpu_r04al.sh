#!/bin/bash
# Persistent band form with its loop-invariant hoisting cut (kernarg + thread index laundered per window, band TU
# built with -mllvm -disable-machine-licm; scripts/_variants/lib_nolicm.so) against the in-tree library:
# per-iteration speed at equal durations, then the bench.
set -o pipefail
O=gpurun_out/r04al; mkdir -p $O
V=scripts/_variants/lib_nolicm.so
for lib in base nolicm; do
  for q in 1 0; do
    if [ $lib = base ]; then L=; else L=$V; fi
    echo "== $lib" >> $O/probe.log
    DVH_LIB=$L DVH_BAND_QUEUE=$q timeout -k 10 300 python -u scripts/probe_band_queue.py 5000 1024 >> $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
  done
done
grep "queue=\|==" $O/probe.log
for r in 1 2; do
  for lib in base nolicm; do
    if [ $lib = base ]; then L=; else L=$V; fi
    echo "== ${lib}_q1" >> $O/ab.log
    DVH_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
  done
done
python scripts/ab_summary.py $O/ab.log

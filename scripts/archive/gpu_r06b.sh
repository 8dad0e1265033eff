#!/bin/bash
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
for L in cur roundonly f32f0; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 120 python -u scripts/probe_t2.py 2 || exit 1
  DVH_BAND_QUEUE=0 timeout -k 10 120 python -u scripts/probe_t2.py 2 || exit 1
done

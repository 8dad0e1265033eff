#!/bin/bash
# Band kernel iteration anatomy: fixed-iteration speed (default build) and per-wave segment cycles (probe build).
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 200 python -u scripts/probe_band_queue.py 5000 1024 > $O/queue.log 2>&1 || { echo "queue probe failed"; tail -20 $O/queue.log; exit 1; }
cat $O/queue.log
DVH_LIB=scripts/_variants/lib_probe.so timeout -k 10 200 python -u scripts/probe_band_latency.py 5000 1024 > $O/latency.log 2>&1 || { echo "latency probe failed"; tail -20 $O/latency.log; exit 1; }
cat $O/latency.log

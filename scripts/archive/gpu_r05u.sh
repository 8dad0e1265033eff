#!/bin/bash
# Inlined KKT helpers in the ICE form and the chain (config 3) kernel vs out of line (lib_kold).
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 120 python -u scripts/probe_band_queue.py 1000 1024 config5 > $O/ice_inl.log 2>&1 || { echo "ice inl failed"; tail -20 $O/ice_inl.log; exit 1; }
DVH_LIB=scripts/_variants/lib_kold.so timeout -k 10 120 python -u scripts/probe_band_queue.py 1000 1024 config5 > $O/ice_old.log 2>&1 || { echo "ice old failed"; tail -20 $O/ice_old.log; exit 1; }
grep -H queue $O/ice_*.log | cut -c1-150
timeout -k 10 200 python -u scripts/probe_config3_opts.py dcm '{}' > $O/c3_inl.log 2>&1 || { echo "c3 inl failed"; tail -20 $O/c3_inl.log; exit 1; }
DVH_LIB=scripts/_variants/lib_kold.so timeout -k 10 200 python -u scripts/probe_config3_opts.py dcm '{}' > $O/c3_old.log 2>&1 || { echo "c3 old failed"; tail -20 $O/c3_old.log; exit 1; }
grep -H dcm $O/c3_*.log | cut -c1-200

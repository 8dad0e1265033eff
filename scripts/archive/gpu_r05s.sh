#!/bin/bash
# KKT check helpers inlined (DVH_KKT_INLINE=1) vs out of line: check schedules at a fixed iteration count.
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 200 python -u scripts/probe_check_cost.py 5000 1024 > $O/cost_noinl.log 2>&1 || { echo "noinl failed"; tail -20 $O/cost_noinl.log; exit 1; }
DVH_LIB=scripts/_variants/lib_kinl.so timeout -k 10 200 python -u scripts/probe_check_cost.py 5000 1024 > $O/cost_inl.log 2>&1 || { echo "inl failed"; tail -20 $O/cost_inl.log; exit 1; }
paste <(grep check_every $O/cost_noinl.log | cut -c1-100) <(grep check_every $O/cost_inl.log | cut -c60-100)

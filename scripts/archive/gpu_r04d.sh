#!/bin/bash
# Team kernel: wave 0's wait times per workgroup (tau partials / boundary hop) and the poll loop with s_sleep.
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
for v in ctime csleep1 csleep4; do
  echo "== $v" >> $O/probe_chain.log
  DVH_CHAIN_PROBE_DUMP=1 DVH_LIB=scripts/_variants/lib_$v.so timeout -k 10 240 python -u scripts/probe_chain.py --iters 8192 da dcm >> $O/probe_chain.log 2>&1 || { echo "$v failed"; tail -20 $O/probe_chain.log; exit 1; }
done
grep -c PROBE $O/probe_chain.log

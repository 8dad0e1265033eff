#!/bin/bash
# Team-kernel iteration anatomy: base vs no tau exchange vs no exchange at all (timing probes, wrong results).
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
for v in cbase cnoxchg cnohop; do
  echo "== $v" >> $O/probe_chain.log
  DVH_LIB=scripts/_variants/lib_$v.so timeout -k 10 240 python -u scripts/probe_chain.py --iters 8192 da dcm_nopv dcm year64 >> $O/probe_chain.log 2>&1 || { echo "$v failed"; tail -20 $O/probe_chain.log; exit 1; }
done
grep -v Warn $O/probe_chain.log | cut -c1-160
# config-5 band-ICE form: LDS relief flags (2 costs, 4 images in the workspace, 1 anchors) vs spills; alternating
for r in 1 2; do
  for v in ice0 ice2 ice5 ice7; do
    echo "== $v" >> $O/ab_ice.log
    DVH_LIB=scripts/_variants/lib_$v.so timeout -k 10 300 python -u bench_configs.py --only 5 --c5-scenarios 500 --c5-years 10 --c5-batch-years 10 --reps 2 --sample 8 >> $O/ab_ice.log 2>&1 || { echo "$v failed"; tail -20 $O/ab_ice.log; exit 1; }
  done
done
grep -E "^==|windows_per_s" $O/ab_ice.log | cut -c1-250

#!/bin/bash
# Compiler options on the chain (config 3) and ELL / generic (market days) units (ab_libs/lib_<v>.so), same box
set -o pipefail
O=gpurun_out/r05zj; mkdir -p $O
r() {
  if [ $1 = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$1.so; fi
  timeout -k 10 300 python -u bench_configs.py --only $2 --sample 0 > $O/cfg_$1_$2.log 2>&1 || { echo "$1 $2 failed"; tail -20 $O/cfg_$1_$2.log; exit 1; }
  grep '^{' $O/cfg_$1_$2.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$1', d['config'], d.get('schedule'), d.get('wall_ms'), d.get('iters_mean'))"
}
r cur 3 && r chain_nolicm 3 && r chain_nounclust 3 && r chain_bias100 3 && r cur 6 && r kern_nolicm 6 && r cur 3

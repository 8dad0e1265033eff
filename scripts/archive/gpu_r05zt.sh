#!/bin/bash
# Team kernel polls with s_sleep back-off (DVH_CHAIN_POLL_SLEEP, ab_libs/lib_sleep<n>.so) vs spinning: configs 3 and medium
set -o pipefail
O=gpurun_out/r05zt; mkdir -p $O
for L in cur sleep0 sleep1 sleep2 cur; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 400 python -u bench_configs.py --only 3,7 --sample 0 > $O/c_$L.log 2>&1 || { echo "$L failed"; tail -20 $O/c_$L.log; exit 1; }
  echo $L $(grep '^{' $O/c_$L.log | python -c "
import sys,json
print(' '.join(str(json.loads(l).get('wall_ms')) for l in sys.stdin))")
done

#!/bin/bash
# ELL / generic unit (no machine LICM) with the primal-weight update out of line: market days and POI windows, same box
set -o pipefail
O=gpurun_out/r05zza; mkdir -p $O
for L in cur k_pwout cur k_pwout; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench_configs.py --only 6 --sample 0 > $O/c_$L.log 2>&1 || { echo "$L failed"; tail -20 $O/c_$L.log; exit 1; }
  echo $L $(grep '^{' $O/c_$L.log | python -c "
import sys,json
print(' '.join(str(json.loads(l).get('wall_ms')) for l in sys.stdin))")
done

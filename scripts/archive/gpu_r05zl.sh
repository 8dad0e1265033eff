#!/bin/bash
# Chain unit (no machine LICM) with further scheduler options: config 3, same box
set -o pipefail
O=gpurun_out/r05zl; mkdir -p $O
for L in cur c_trk c_nouncl c_nocluster c_maxilp c_nopostrasink cur; do
  if [ $L = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench_configs.py --only 3 --sample 0 > $O/c3_$L.log 2>&1 || { echo "$L failed"; tail -20 $O/c3_$L.log; exit 1; }
  echo $L $(grep '^{' $O/c3_$L.log | python -c "
import sys,json
print(' '.join(str(json.loads(l).get('wall_ms')) for l in sys.stdin))")
done

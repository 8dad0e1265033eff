#!/bin/bash
# ICE form: rows 2.. of the DCM/ICE row block moved after the second barrier on waves 1-3 (DVH_BAND_LATE_ICE), A/B on config 5
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
for L in cur lateice cur lateice; do
  export DVH_LIB=ab_libs/lib_$L.so
  timeout -k 10 400 python -u bench_configs.py --only 5 --sample 0 > $O/c5_$L.log 2>&1 || { echo "$L c5 failed"; tail -20 $O/c5_$L.log; exit 1; }
  echo "$L c5 $(grep '"config5"' $O/c5_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d.get('max_primal_res_rel'))")"
done

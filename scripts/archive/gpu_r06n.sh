#!/bin/bash
# team-kernel anatomy on the round-6 sources: fixed 8,192 iterations (scripts/probe_chain.py), current / no tau exchange /
# no exchange at all (probe builds, wrong results, timing only)
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
for L in cur cnoxchg cnohop; do
  export DVH_LIB=ab_libs/lib_$L.so
  timeout -k 10 300 python -u scripts/probe_chain.py --iters 8192 da dcm year64 > $O/probe_$L.log 2>&1 || { echo "$L failed"; tail -20 $O/probe_$L.log; exit 1; }
  echo "== $L"; grep '^{' $O/probe_$L.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['variant'], d['windows'], d['iters'], d['pdhg_ms'], d['us_per_iter'])"
done

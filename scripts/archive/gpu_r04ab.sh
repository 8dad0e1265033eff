#!/bin/bash
# A/B of the objective gate's dual-residual term: config 5 and the bench, main library (term on) vs lib_rdx0 (off).
set -o pipefail
O=gpurun_out/r04ab; mkdir -p $O
for r in 1 2; do
  for v in main rdx0; do
    L=""; [ $v = rdx0 ] && L=scripts/_variants/lib_rdx0.so
    echo "== $v" >> $O/c5.log
    DVH_LIB=$L timeout -k 10 300 python -u bench_configs.py --only 5 --c5-scenarios 500 --c5-years 10 >> $O/c5.log 2>&1 || { echo "c5 failed"; tail -20 $O/c5.log; exit 1; }
    echo "== $v" >> $O/ab.log
    DVH_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
  done
done
python scripts/ab_summary.py $O/ab.log
python - <<'PY'
import json
v=None
for line in open('gpurun_out/r04ab/c5.log'):
    if line.startswith('=='): v=line.strip()
    elif line.startswith('{'):
        j=json.loads(line); print(v, j['windows_per_s'], j['solve_ms_total'], j['iters_mean'])
PY

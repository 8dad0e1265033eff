#!/bin/bash
# Persistent work-queue band kernel (DVH_BAND_QUEUE=2) x warm-phase launch order (seed predictor), and config 5.
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
for r in 1 2; do
  for q in 0 2; do
    for v in 0 1; do
      echo "== q${q}_order${v}" >> $O/ab.log
      DVH_SWEEP_ORDER=$v DVH_BAND_QUEUE=$q timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
    done
  done
done
python scripts/ab_summary.py $O/ab.log
for q in 0 2; do
  echo "== c5_q$q" >> $O/c5.log
  DVH_BAND_QUEUE=$q timeout -k 10 300 python -u bench_configs.py --only 5 --c5-scenarios 500 --c5-years 10 >> $O/c5.log 2>&1 || { echo "c5 failed"; tail -20 $O/c5.log; exit 1; }
done
grep -E '^==|^\{' $O/c5.log | cut -c1-80
python - <<'PY'
import json
v=None
for line in open('gpurun_out/r04u/c5.log'):
    if line.startswith('=='): v=line.split()[1]
    elif line.startswith('{'):
        j=json.loads(line); print(v, j['windows_per_s'], j['solve_ms_total'])
PY

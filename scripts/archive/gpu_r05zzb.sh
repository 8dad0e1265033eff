#!/bin/bash
# Seed-phase check schedule (bench.py --check-every / --kkt-every act on the cold seed phase; the warm phase keeps
# sweep.WARM_OPTIONS): bench, same box
set -o pipefail
O=gpurun_out/r05zzb; mkdir -p $O
for cfg in "0 0" "64 0" "64 2" "32 2" "16 0" "0 0"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 6 --warmup 2 --check-every $1 --kkt-every $2 > $O/b_$1_$2.log 2>&1 || { echo "$cfg failed"; tail -20 $O/b_$1_$2.log; exit 1; }
  echo "check $1 kkt $2" $(tail -1 $O/b_$1_$2.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); s=d['schedule']; print(d['value'], d['ms_per_step'], d['iters_mean'], s['iters_mean_seed'], s['iters_mean_warm'], d['max_primal_res_rel'])")
done

#!/bin/bash
# Seeded schedule parameters on the current kernel: seed stride, blend size, blend-weight power (bench.py, same box)
set -o pipefail
O=gpurun_out/r05zo; mkdir -p $O
for cfg in "32 4 1" "24 4 1" "16 4 1" "48 4 1" "32 6 1" "32 8 1" "32 4 2" "32 4 0.5" "32 4 1"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 6 --warmup 2 --seed-stride $1 --blend $2 --blend-power $3 > $O/b_$1_$2_$3.log 2>&1 || { echo "$cfg failed"; tail -20 $O/b_$1_$2_$3.log; exit 1; }
  echo "stride $1 blend $2 power $3" $(tail -1 $O/b_$1_$2_$3.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); s=d['schedule']; print(d['value'], d['ms_per_step'], d['iters_mean'], s['iters_mean_seed'], s['iters_mean_warm'], d['max_primal_res_rel'])")
done

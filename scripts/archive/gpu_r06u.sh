#!/bin/bash
# warm-phase restart-check period re-tuned on the current band kernel (bench steps on one box, two rounds)
set -o pipefail
O=gpurun_out/r06u; mkdir -p $O
run() {  # name warm
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 --warm-options "$2" > $O/bench_$1.log 2>&1 || { echo "$1 bench failed"; tail -20 $O/bench_$1.log; exit 1; }
  echo $1 $(tail -1 $O/bench_$1.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); s=d['schedule']; print(d['value'], d['ms_per_step'], d['iters_mean'], s['iters_mean_seed'], s['iters_mean_warm'], d['max_primal_res_rel'])")
}
for r in 1 2; do
  run base$r '{"check_every": 64, "kkt_every": 1, "kkt_predict": 4}'
  run c56_$r '{"check_every": 56, "kkt_every": 1, "kkt_predict": 4}'
  run c72_$r '{"check_every": 72, "kkt_every": 1, "kkt_predict": 4}'
  run c80_$r '{"check_every": 80, "kkt_every": 1, "kkt_predict": 4}'
done

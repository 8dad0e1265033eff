#!/bin/bash
# warm-phase restart-check period around 72 (robustness of the r06u result), bench steps on one box
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
run() {  # name warm
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 --warm-options "$2" > $O/bench_$1.log 2>&1 || { echo "$1 bench failed"; tail -20 $O/bench_$1.log; exit 1; }
  echo $1 $(tail -1 $O/bench_$1.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); s=d['schedule']; print(d['value'], d['ms_per_step'], d['iters_mean'], s['iters_mean_seed'], s['iters_mean_warm'], d['max_primal_res_rel'])")
}
run c64 '{"check_every": 64, "kkt_every": 1, "kkt_predict": 4}'
run c68 '{"check_every": 68, "kkt_every": 1, "kkt_predict": 4}'
run c72 '{"check_every": 72, "kkt_every": 1, "kkt_predict": 4}'
run c76 '{"check_every": 76, "kkt_every": 1, "kkt_predict": 4}'
run c72p2 '{"check_every": 72, "kkt_every": 1, "kkt_predict": 2}'
run c72k2 '{"check_every": 72, "kkt_every": 2, "kkt_predict": 4}'

#!/bin/bash
# The seeded schedule's check options re-tuned for the cheaper KKT check (batched factor loads): warm-phase restart
# period and KKT gate, cold-phase gate; bench steps on one box
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
run() {  # name warm seed
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 --warm-options "$2" --seed-options "$3" > $O/bench_$1.log 2>&1 || { echo "$1 bench failed"; tail -20 $O/bench_$1.log; exit 1; }
  echo $1 $(tail -1 $O/bench_$1.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); s=d['schedule']; print(d['value'], d['ms_per_step'], d['iters_mean'], s['iters_mean_seed'], s['iters_mean_warm'], d['max_primal_res_rel'])")
}
run base '{"check_every": 64, "kkt_every": 1, "kkt_predict": 4}' '{"kkt_predict": 4}'
run w_p2 '{"check_every": 64, "kkt_every": 1, "kkt_predict": 2}' '{"kkt_predict": 4}'
run w_p8 '{"check_every": 64, "kkt_every": 1, "kkt_predict": 8}' '{"kkt_predict": 4}'
run w_c48 '{"check_every": 48, "kkt_every": 1, "kkt_predict": 4}' '{"kkt_predict": 4}'
run w_c96 '{"check_every": 96, "kkt_every": 1, "kkt_predict": 4}' '{"kkt_predict": 4}'
run s_k2 '{"check_every": 64, "kkt_every": 1, "kkt_predict": 4}' '{"kkt_predict": 4, "kkt_every": 2}'
run s_c64 '{"check_every": 64, "kkt_every": 1, "kkt_predict": 4}' '{"kkt_predict": 4, "check_every": 64, "kkt_every": 1}'
run base2 '{"check_every": 64, "kkt_every": 1, "kkt_predict": 4}' '{"kkt_predict": 4}'
echo all done

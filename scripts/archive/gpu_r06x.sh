#!/bin/bash
# warm check period 72: certification dump (seeded, every bench window), config 5, bench line
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 400 python -u scripts/certify_dump.py --label c72 --blend 4 --no-cold > $O/certify.log 2>&1 || { echo "dump failed"; tail -20 $O/certify.log; exit 1; }
tail -2 $O/certify.log
timeout -k 10 400 python -u bench_configs.py --only 5 --sample 0 > $O/c5.log 2>&1 || { echo "c5 failed"; tail -20 $O/c5.log; exit 1; }
echo "c5 $(grep '"config5"' $O/c5.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['windows_per_s'], d['solve_ms_total'], d['iters_mean'])")"
timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench.log 2>&1 || { echo "bench failed"; exit 1; }
echo bench $(tail -1 $O/bench.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['iters_mean'], d['kernel_ms'], d['roofline']['frac'])")

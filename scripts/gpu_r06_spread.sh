#!/bin/bash
# run-to-run spread of the driver's bench command on one box (3 runs, --no-cpu to keep it short)
set -o pipefail
O=gpurun_out/r06_spread; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_$r.log 2>&1 || { echo "bench $r failed"; exit 1; }
  tail -1 $O/bench_$r.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('run', $r, d['value'], d['ms_per_step'], d['kernel_ms']['pdhg'], r['frac'], r['achieved'])"
done

#!/bin/bash
# Bit-identity bisection: SHA-256 of the bench batch's outputs after a seeded step, per library build
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
for L in cur cur2 hdiv0 widths pf0 all0 r5src r5; do
  if [ $L = cur ] || [ $L = cur2 ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 2 --warmup 0 --sha > $O/sha_$L.log 2>&1 || { echo "$L sha failed"; tail -20 $O/sha_$L.log; exit 1; }
  echo $L $(tail -1 $O/sha_$L.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['iters_mean'], d['max_primal_res_rel'], d['outputs_sha256'])")
done

#!/bin/bash
# Same-box A/B of library builds on the default bench (no CPU leg, no cold reference), alternating runs.
# Usage (on the GPU box): scripts/ab_bench.sh <out> <reps> <name> [<name> ...]   (scripts/_variants/lib_<name>.so)
O=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for v in "$@"; do
    echo "== $v" >> $O
    DVH_LIB=scripts/_variants/lib_$v.so timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 3 >> $O 2>&1 || exit 1
  done
done

#!/bin/bash
# Same-box A/B of the band kernel's in-kernel scaling of the band windows (lib_self) against HEAD (lib_base): bench
# throughput, iterations / objectives on a config-4 sample, and FETCH_SIZE / WRITE_SIZE of one bench step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r03m
mkdir -p $O
cd $R
bash scripts/ab_bench.sh $O/ab_self_bench.log 2 base self || exit 1
timeout -k 10 300 python -u scripts/ab_variants.py 2000 scripts/_variants/lib_base.so scripts/_variants/lib_self.so \
  > $O/ab_self_variants.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in base self; do
  for c in FETCH_SIZE WRITE_SIZE; do
    DVH_LIB=$R/scripts/_variants/lib_$v.so timeout -s KILL 240 rocprofv3 --pmc $c -d $O/pmc_${v}_$c -o run \
      --output-format csv -- python3 $R/bench.py --no-cpu --no-cold-ref --steps 1 --warmup 0 > $O/pmc_${v}_$c.log 2>&1 \
      || { echo "pmc $v $c failed"; exit 1; }
  done
done
echo done

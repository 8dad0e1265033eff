#!/bin/bash
# HBM bytes of the bench's band kernel by check schedule at a fixed iteration count (FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05zs; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for sch in "1024 1000" "64 1000" "64 1"; do
  set -- $sch
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c -d $O/${c}_$1_$2 -o run --output-format csv -- python3 $R/scripts/probe_traffic_sched.py $1 $2 > $O/${c}_$1_$2.log 2>&1 || { echo "$c $sch failed"; tail -5 $O/${c}_$1_$2.log; exit 1; }
  done
done
echo done

#!/bin/bash
# On the GPU box: kernel-trace stats of the default bench command, then two PMC passes (FETCH_SIZE, WRITE_SIZE;
# counters in their own runs, no other tracing).  Usage: scripts/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py \
  > $O/bench_trace.log 2>&1 || { echo "trace run failed: $?"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 \
  > $O/pmc_fetch.log 2>&1 || { echo "fetch pass failed: $?"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 \
  > $O/pmc_write.log 2>&1 || { echo "write pass failed: $?"; exit 1; }
echo done

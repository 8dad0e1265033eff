#!/bin/bash
# On the GPU box: kernel-trace stats of the default bench command, then two PMC passes (FETCH_SIZE, WRITE_SIZE;
# counters in their own runs, no other tracing) over exactly one bench step (no cold reference solve), then
# profiles/pdhg_traffic.json from them.  Usage: scripts/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cold-ref --no-cpu \
  > $O/bench_trace.log 2>&1 || { echo "trace run failed: $?"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-cold-ref --steps 1 --warmup 0 \
  > $O/pmc_fetch.log 2>&1 || { echo "fetch pass failed: $?"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-cold-ref --steps 1 --warmup 0 \
  > $O/pmc_write.log 2>&1 || { echo "write pass failed: $?"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d $O/sq -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-cold-ref --steps 1 --warmup 0 \
  > $O/pmc_sq.log 2>&1 || { echo "sq pass failed: $?"; exit 1; }
python3 $R/scripts/pmc_valu.py $O/sq 120000 $O/pdhg_valu.json > $O/valu.log 2>&1 || { echo "valu failed"; exit 1; }
python3 $R/scripts/pmc_traffic.py $O/fetch $O/write 120000 $O/pdhg_traffic.json 2 > $O/traffic.log 2>&1 || { echo "traffic failed"; exit 1; }
echo done

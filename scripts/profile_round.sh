#!/bin/bash
# On the GPU box: kernel-trace stats of the default bench command, then PMC passes (each counter group in a run of its
# own, no other tracing) over exactly one bench step (no cold reference solve, no CPU leg): FETCH_SIZE, WRITE_SIZE
# (HBM bytes), FP64 / VALU instruction counts, and the issue / wait picture; then profiles-ready JSON
# (pdhg_traffic.json, pdhg_valu.json, keyed to the kernel sources).  Usage: scripts/profile_round.sh <tag> [windows]
set -o pipefail
TAG=${1:-r02}
WIN=${2:-120000}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --no-cold-ref"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B --steps 5 --warmup 1 \
  > $O/bench_trace.log 2>&1 || { echo "trace run failed: $?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B --steps 1 --warmup 0 \
  > $O/pmc_fetch.log 2>&1 || { echo "fetch pass failed: $?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B --steps 1 --warmup 0 \
  > $O/pmc_write.log 2>&1 || { echo "write pass failed: $?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $O/sq -o run --output-format csv -- $B --steps 1 --warmup 0 \
  > $O/pmc_sq.log 2>&1 || { echo "sq pass failed: $?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/sq2 -o run --output-format csv -- $B --steps 1 --warmup 0 \
  > $O/pmc_sq2.log 2>&1 || { echo "sq2 pass failed: $?"; exit 1; }
python3 $R/scripts/pmc_valu.py $O/sq $WIN $O/pdhg_valu.json $O/sq2 > $O/valu.log 2>&1 || { echo "valu failed"; exit 1; }
python3 $R/scripts/pmc_traffic.py $O/fetch $O/write $WIN $O/pdhg_traffic.json 2 > $O/traffic.log 2>&1 || { echo "traffic failed"; exit 1; }
echo done

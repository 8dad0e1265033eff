#!/bin/bash
# On the GPU box: SQ counter passes (own runs, kernel-trace free) over one solve of a config-4 sample.
# Usage: scripts/pmc_sq.sh <tag> [scenarios]
set -o pipefail
TAG=${1:-sq}; S=${2:-256}; [ -n "$3" ] && export DVH_AB_LIB=$(cd "$(dirname "$3")" && pwd)/$(basename "$3")
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 $R/scripts/prof_kernel.py $S \
    > $O/p$i.log 2>&1 || { echo "pass $i failed: $?"; tail -5 $O/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/p1 $O/p2 > $O/summary.txt && cat $O/summary.txt

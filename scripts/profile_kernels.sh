#!/bin/bash
# On the GPU box: kernel-trace + PMC passes (FETCH_SIZE, WRITE_SIZE, FP64/VALU group, each a run of its own) of the
# config-3 long team (pdhg_chain_kernel, DCM + PV) and the config-5 ICE band form; JSON per kernel via pmc_kernel.py.
# Usage: scripts/profile_kernels.sh <tag>
set -o pipefail
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
for job in c3 c5; do
  if [ $job = c3 ]; then C="python3 $R/scripts/prof_config3.py dcm"; K=pdhg_chain_kernel; else C="python3 $R/scripts/prof_config5.py 100"; K="pdhg_band_kernel<768, 1, true"; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/${job}_trace -o run --output-format csv -- $C > $O/${job}_trace.log 2>&1 || { echo "$job trace failed: $?"; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/${job}_fetch -o run --output-format csv -- $C > $O/${job}_fetch.log 2>&1 || { echo "$job fetch failed: $?"; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/${job}_write -o run --output-format csv -- $C > $O/${job}_write.log 2>&1 || { echo "$job write failed: $?"; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $SQ -d $O/${job}_sq -o run --output-format csv -- $C > $O/${job}_sq.log 2>&1 || { echo "$job sq failed: $?"; exit 1; }
  python3 $R/scripts/pmc_kernel.py "$K" $O/${job}_trace $O/${job}_pmc.json $job $O/${job}_fetch $O/${job}_write $O/${job}_sq > $O/${job}_pmc.log 2>&1 || { echo "$job summary failed"; cat $O/${job}_pmc.log; exit 1; }
  echo "$job done"
done

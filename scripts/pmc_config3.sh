#!/bin/bash
# One PMC counter pass over one config-3 cold solve (after a warm-up) on the GPU box.  (Round 3's exit crash under the
# profiler came from the team kernel's cooperative launch, now an ordinary launch: profiles/r04a_chain_exit_crash.txt.)
# Usage: scripts/pmc_config3.sh <tag> <FETCH_SIZE|WRITE_SIZE> [variant]
set -o pipefail
TAG=${1:-r03}; C=${2:-FETCH_SIZE}; V=${3:-dcm_nopv}
R=$(pwd); O=$R/gpurun_out/prof_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc $C -d $O/c3_$C -o run --output-format csv -- python3 $R/scripts/prof_config3.py $V > $O/c3_$C.log 2>&1
echo "rc=$?"
grep '^{' $O/c3_$C.log
find $O/c3_$C -name "*counter_collection.csv" | head -2

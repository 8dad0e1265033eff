#!/bin/bash
# Kernel traces of the mixed batch (scripts/mixed_batch.py) with the previous and the current library.
set -o pipefail
TAG=${1:-cascade_trace}; OLD=$2
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
DVH_LIB=$R/$OLD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/old -o run --output-format csv -- python3 $R/scripts/mixed_batch.py > $O/old.log 2>&1 || { echo "old failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/new -o run --output-format csv -- python3 $R/scripts/mixed_batch.py > $O/new.log 2>&1 || { echo "new failed"; exit 1; }
echo ok

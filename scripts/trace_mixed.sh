#!/bin/bash
# Kernel trace of the mixed batch (scripts/mixed_batch.py) with the current library.
set -o pipefail
TAG=${1:-mixed_trace}
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/new -o run --output-format csv -- python3 $R/scripts/mixed_batch.py > $O/new.log 2>&1 || { echo "trace failed"; tail -5 $O/new.log; exit 1; }
echo ok

#!/bin/bash
# Round-3 profiles on the GPU box: HIP API trace of the cascade's host waits (band-only batch), then config 3 (DCM + PV,
# long team): kernel trace + FETCH_SIZE / WRITE_SIZE PMC passes (one counter per pass).  Config 3 last.
set -o pipefail
TAG=${1:-r03}
R=$(pwd); O=$R/gpurun_out/prof_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-trace --stats -d $O/syncs -o run --output-format csv -- python3 $R/scripts/prof_syncs.py > $O/syncs.log 2>&1 || { echo "syncs trace failed"; tail -5 $O/syncs.log; exit 1; }
grep '^{' $O/syncs.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/c3trace -o run --output-format csv -- python3 $R/scripts/prof_config3.py > $O/c3trace.log 2>&1 || { echo "c3 trace failed"; tail -5 $O/c3trace.log; exit 1; }
grep '^{' $O/c3trace.log
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/c3fetch -o run --output-format csv -- python3 $R/scripts/prof_config3.py > $O/c3fetch.log 2>&1 || { echo "c3 fetch failed"; tail -5 $O/c3fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/c3write -o run --output-format csv -- python3 $R/scripts/prof_config3.py > $O/c3write.log 2>&1 || { echo "c3 write failed"; tail -5 $O/c3write.log; exit 1; }
echo done

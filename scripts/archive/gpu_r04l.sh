#!/bin/bash
# Round-4 profiles on the final band-kernel sources: kernel trace + stats of the default bench, PMC passes (HBM bytes,
# FP64 / VALU counts, issue / wait picture) over one bench step, and the config-3 team kernel's trace (exits 0 now).
set -o pipefail
bash scripts/profile_round.sh r04l || exit 1
R=$(pwd); O=$R/gpurun_out/prof_r04l
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/c3trace -o run --output-format csv -- python3 $R/scripts/prof_config3.py dcm > $O/c3trace.log 2>&1
echo "c3 trace rc=$?"
grep '^{' $O/c3trace.log | cut -c1-200

#!/bin/bash
# pw_update_general inlined (DVH_PW_INLINE=1) vs a call: quick A/B over the band forms, market days, config 3.
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 200 python -u scripts/ab_quick.py base > $O/base.log 2>&1 || { echo "base failed"; tail -20 $O/base.log; exit 1; }
DVH_LIB=scripts/_variants/lib_pwinl.so timeout -k 10 200 python -u scripts/ab_quick.py pw_inline > $O/pwinl.log 2>&1 || { echo "pwinl failed"; tail -20 $O/pwinl.log; exit 1; }
grep -h '^{' $O/base.log $O/pwinl.log

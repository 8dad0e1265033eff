#!/bin/bash
# Full-population certification dump of the bench schedule with blended warm starts (4 nearest seeds): every window's
# objective / status / iterations, seeded and all-cold; compared with HiGHS on the host (scripts/certify_highs.py).
set -o pipefail
timeout -k 10 400 python -u scripts/certify_dump.py --label r04j --blend 4 > gpurun_out/r04j_certify_dump.log 2>&1 || { echo "dump failed"; tail -20 gpurun_out/r04j_certify_dump.log; exit 1; }
tail -4 gpurun_out/r04j_certify_dump.log

#!/bin/bash
# Certification dumps on the box-form / persistent kernel: default options (seeded + cold), and eps_obj 7e-7 seeded.
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 300 python -u scripts/certify_dump.py --label r04w --blend 4 > $O/certify.log 2>&1 || { echo "dump failed"; tail -20 $O/certify.log; exit 1; }
timeout -k 10 300 python -u scripts/certify_dump.py --label r04w_eobj7 --blend 4 --no-cold --opt eps_obj=7e-7 >> $O/certify.log 2>&1 || { echo "dump2 failed"; tail -20 $O/certify.log; exit 1; }
grep -E "seeded|cold|wrote" $O/certify.log

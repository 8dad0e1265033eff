#!/bin/bash
set -o pipefail
for W in 1 64 65 128 1000; do
unset DVH_LIB; AB_WARM_ITERS=$W timeout -k 10 200 python -u scripts/ab_arrays.py run cur 200 warm || exit 1
AB_WARM_ITERS=$W DVH_LIB=ab_libs/lib_pf0.so timeout -k 10 200 python -u scripts/ab_arrays.py run pf0 200 warm || exit 1
echo "== warm max_iters $W"; python scripts/ab_arrays.py compare cur pf0
done
rm -f gpurun_out/ab_*.npz

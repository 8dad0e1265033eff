#!/bin/bash
# Dispatch probe (synthetic) + the band kernel's persistent work-queue form (DVH_BAND_QUEUE=2): tests, bench A/B.
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 90 scripts/_variants/probe_dispatch 30000 > $O/probe.log 2>&1 || { echo "probe failed rc=$?"; cat $O/probe.log; exit 1; }
cat $O/probe.log
DVH_BAND_QUEUE=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_band_scaling.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests q2 failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 0 2; do
    echo "== queue_$v" >> $O/ab.log
    DVH_SWEEP_ORDER=0 DVH_BAND_QUEUE=$v timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
  done
done
python scripts/ab_summary.py $O/ab.log

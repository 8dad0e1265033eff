#!/bin/bash
# Band-kernel work distribution A/B: static blockIdx mapping (0), counter mapping in start order (1), persistent
# work-queue loop (2); and the static mapping with the previous step's own counts as launch order (ceiling).
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_band_scaling.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
DVH_BAND_QUEUE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_band_scaling.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread >> $O/tests.log 2>&1 || { echo "tests q2 failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 0 1; do
    echo "== queue_$v" >> $O/ab.log
    DVH_SWEEP_ORDER=0 DVH_BAND_QUEUE=$v timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
  done
  echo "== prev_0" >> $O/ab.log
  DVH_SWEEP_ORDER=prev DVH_BAND_QUEUE=0 timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
done
python scripts/ab_summary.py $O/ab.log

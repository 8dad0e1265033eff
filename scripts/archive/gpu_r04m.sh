#!/bin/bash
# Box form (dvh_band.hip BOX): band / config / parity tests, then a same-box bench A/B against the plain form.
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_band_scaling.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    echo "== box_$v" >> $O/ab.log
    DVH_BAND_BOX=$v timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 5 >> $O/ab.log 2>&1 || { echo "bench failed"; tail -20 $O/ab.log; exit 1; }
  done
done
python scripts/ab_summary.py $O/ab.log 2>/dev/null || grep -E '^==|^\{' $O/ab.log | cut -c1-300

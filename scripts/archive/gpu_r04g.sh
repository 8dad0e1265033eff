#!/bin/bash
# Band kernel: per-wave tau sums (default) vs wave 0 reducing every lane's partial (round 3), same-box A/B on the bench;
# then the band / sweep GPU tests on the default build.
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
bash scripts/ab_bench.sh $O/ab_tw.log 2 tw1 tw0 || { echo "ab failed"; tail -30 $O/ab_tw.log; exit 1; }
python scripts/ab_summary.py $O/ab_tw.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_band_scaling.py tests/test_sweep.py tests/test_gpu_cascade.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log

#!/bin/bash
# Persistent band form in its own translation unit without machine LICM (dvh_band_persist.hip): GPU suite, smoke,
# equal-duration probe, bench, PMC passes of the bench (new source key), configs.
set -o pipefail
O=gpurun_out/r04am; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
for q in 1 0; do
  DVH_BAND_QUEUE=$q timeout -k 10 300 python -u scripts/probe_band_queue.py 5000 1024 >> $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
done
grep "queue=" $O/probe.log | cut -c1-110
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300
scripts/profile_round.sh r04am || exit 1
timeout -k 10 600 python -u bench_configs.py --only 1,2,3,5 --sample 16 > $O/bench_configs.log 2>&1 || { echo "configs failed"; tail -30 $O/bench_configs.log; exit 1; }
grep '^{' $O/bench_configs.log | cut -c1-200

#!/bin/bash
# Final round-5 sources (final: + chain KKT helpers out of line): GPU suite + smoke + certification dump, bench-step trace + PMC
# passes (profiles/pdhg_*.json keyed to the sources), the bench line, config-3 / config-5 kernel PMC, every config.
set -o pipefail
O=gpurun_out/r05z5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u scripts/certify_dump.py --label r05z5 --blend 4 > $O/certify.log 2>&1 || { echo "dump failed"; tail -20 $O/certify.log; exit 1; }
bash scripts/profile_round.sh r05z5 > $O/profile_round.log 2>&1 || { echo "profile_round failed"; tail -20 $O/profile_round.log; exit 1; }
cp gpurun_out/prof_r05z5/pdhg_valu.json gpurun_out/prof_r05z5/pdhg_traffic.json profiles/
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
bash scripts/profile_kernels.sh r05z5 > $O/profile_kernels.log 2>&1 || { echo "profile_kernels failed"; tail -20 $O/profile_kernels.log; exit 1; }
timeout -k 10 600 python -u bench_configs.py --only 1,2,3,5 > $O/bench_configs_1235.log 2>&1 || { echo "configs failed"; tail -30 $O/bench_configs_1235.log; exit 1; }
timeout -k 10 600 python -u bench_configs.py --only 6,7,8 > $O/bench_configs_678.log 2>&1 || { echo "configs 678 failed"; tail -30 $O/bench_configs_678.log; exit 1; }
echo all done

#!/bin/bash
# Final round-5 sources: bench-step trace + PMC passes (profiles/pdhg_*.json keyed to the sources), the bench line with
# its roofline, the config-3 / config-5 kernel PMC, and bench_configs over every config.
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
bash scripts/profile_round.sh r05z > $O/profile_round.log 2>&1 || { echo "profile_round failed"; tail -20 $O/profile_round.log; exit 1; }
cp gpurun_out/prof_r05z/pdhg_valu.json gpurun_out/prof_r05z/pdhg_traffic.json profiles/
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
bash scripts/profile_kernels.sh r05z > $O/profile_kernels.log 2>&1 || { echo "profile_kernels failed"; tail -20 $O/profile_kernels.log; exit 1; }
timeout -k 10 600 python -u bench_configs.py --only 1,2,3,5 > $O/bench_configs_1235.log 2>&1 || { echo "configs failed"; tail -30 $O/bench_configs_1235.log; exit 1; }
timeout -k 10 600 python -u bench_configs.py --only 6,7,8 > $O/bench_configs_678.log 2>&1 || { echo "configs 678 failed"; tail -30 $O/bench_configs_678.log; exit 1; }
echo all done

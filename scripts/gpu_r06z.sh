#!/bin/bash
# Round-6 final sources: GPU suite + smoke, certification dump (seeded + cold, every bench window), bench-step trace +
# PMC passes (profiles/pdhg_*.json keyed to the sources and build configuration), the bench line with the driver's
# command, the rocprof summary of that command, config-3 / config-5 kernel PMC, every config.
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
echo "box key $(python -c 'import sys; sys.path[:0]=[".","der-vet_amd"]; import bench; print(bench.source_key())')"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u scripts/certify_dump.py --label r06z --blend 4 > $O/certify.log 2>&1 || { echo "dump failed"; tail -20 $O/certify.log; exit 1; }
tail -3 $O/certify.log
bash scripts/profile_round.sh r06z > $O/profile_round.log 2>&1 || { echo "profile_round failed"; tail -20 $O/profile_round.log; exit 1; }
cp gpurun_out/prof_r06z/pdhg_valu.json gpurun_out/prof_r06z/pdhg_traffic.json profiles/
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/bench_trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/bench_traced.log 2>&1 || { echo "traced bench failed"; tail -20 $GRAFT_REPO_ROOT/$O/bench_traced.log; exit 1; }
cd $GRAFT_REPO_ROOT
bash scripts/profile_kernels.sh r06z > $O/profile_kernels.log 2>&1 || { echo "profile_kernels failed"; tail -20 $O/profile_kernels.log; exit 1; }
timeout -k 10 600 python -u bench_configs.py --only 1,2,3,5 > $O/bench_configs_1235.log 2>&1 || { echo "configs failed"; tail -30 $O/bench_configs_1235.log; exit 1; }
timeout -k 10 600 python -u bench_configs.py --only 6,7,8 > $O/bench_configs_678.log 2>&1 || { echo "configs 678 failed"; tail -30 $O/bench_configs_678.log; exit 1; }
echo all done

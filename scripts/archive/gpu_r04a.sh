#!/bin/bash
# Round 4, first GPU call: the GPU suite on HEAD, the max-ilp scheduler A/B of the band kernel on the bench, the
# self-launched 2-rank (gloo) bench, then the config-3 exit crash under rocprofv3: ordinary launch of the team kernel
# first, the cooperative launch (the round-3 crash) last, each dumping /proc/self/maps.
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash scripts/ab_bench.sh $O/ab_maxilp.log 2 base maxilp || { echo "ab failed"; tail -30 $O/ab_maxilp.log; exit 1; }
python scripts/ab_summary.py $O/ab_maxilp.log
bash scripts/rehearse_2rank.sh r04a_2rank 2000 || exit 1
cd /tmp && export TMPDIR=/tmp
export DVH_CHAIN_LAUNCH=plain DVH_DUMP_MAPS=$R/$O/maps_plain.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/$O/c3plain -o run --output-format csv -- python3 $R/scripts/prof_config3.py dcm > $R/$O/c3plain.log 2>&1
echo "plain rc=$?"; grep '^{' $R/$O/c3plain.log | cut -c1-300
export DVH_CHAIN_LAUNCH=coop DVH_DUMP_MAPS=$R/$O/maps_coop.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/$O/c3coop -o run --output-format csv -- python3 $R/scripts/prof_config3.py dcm > $R/$O/c3coop.log 2>&1
echo "coop rc=$?"; grep '^{' $R/$O/c3coop.log | cut -c1-300
exit 0

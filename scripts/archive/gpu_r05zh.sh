#!/bin/bash
# Battery persistent form built with the AMDGPU register-pressure trackers (ICE form in its own unit without them):
# GPU tests of the band forms, bench and config 5 on the current library, and the trackers tried on the other units
set -o pipefail
O=gpurun_out/r05zh; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band_scaling.py tests/test_gpu_configs.py tests/test_sweep.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
r() {  # r <lib|cur> <only>
  if [ $1 = cur ]; then unset DVH_LIB; else export DVH_LIB=ab_libs/lib_$1.so; fi
  timeout -k 10 300 python -u bench_configs.py --only $2 --sample 0 > $O/cfg_$1_$2.log 2>&1 || { echo "$1 $2 failed"; tail -20 $O/cfg_$1_$2.log; exit 1; }
  grep '^{' $O/cfg_$1_$2.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$1', d['config'], d.get('schedule'), d.get('wall_ms'), d.get('windows_per_s'), d.get('solve_ms_total'), d.get('iters_mean'))"
}
timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 10 --warmup 3 > $O/bench_cur.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 $O/bench_cur.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('cur bench', d['value'], d['ms_per_step'], d['iters_mean'], d['max_primal_res_rel'])"
r cur 5 && r trk_ice 5 && r cur 1,2 && r trk_band 1,2 && r cur 3 && r trk_chain 3 && r cur 6 && r trk_kernels 6 && r cur 5

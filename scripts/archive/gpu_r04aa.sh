#!/bin/bash
# Config 5 A/B: default vs one-workgroup battery pass (DVH_BAND_QUEUE=0) vs the ICE box form (DVH_BAND_BOX=2).
set -o pipefail
O=gpurun_out/r04aa; mkdir -p $O
for r in 1 2; do
  for v in "" "DVH_BAND_QUEUE=0" "DVH_BAND_BOX=2" "DVH_BAND_QUEUE=0 DVH_BAND_BOX=2"; do
    echo "== [$v]" >> $O/c5.log
    env $v timeout -k 10 300 python -u bench_configs.py --only 5 --c5-scenarios 500 --c5-years 10 >> $O/c5.log 2>&1 || { echo "c5 failed"; tail -20 $O/c5.log; exit 1; }
  done
done
python - <<'PY'
import json
v=None
for line in open('gpurun_out/r04aa/c5.log'):
    if line.startswith('=='): v=line.strip()
    elif line.startswith('{'):
        j=json.loads(line); print(v, j['windows_per_s'], j['solve_ms_total'], j['iters_mean'])
PY

#!/bin/bash
# Seeded sweep with blended warm starts: partners (3, 4) and seed stride (24, 32, 48), same box, alternating.
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
for r in 1 2; do
  for cfg in "3 32" "4 32" "4 24" "4 48" "6 32"; do
    set -- $cfg
    echo "== b$1s$2" >> $O/ab_blend.log
    timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 3 --blend $1 --seed-stride $2 >> $O/ab_blend.log 2>&1 || { echo "cfg $cfg failed"; tail -20 $O/ab_blend.log; exit 1; }
  done
done
python - <<'PY'
import json, collections
v=None; res=collections.defaultdict(list)
for l in open("gpurun_out/r04i/ab_blend.log"):
    if l.startswith("=="): v=l.split()[1]
    elif l.startswith("{"):
        j=json.loads(l); res[v].append((j["value"], j["kernel_ms"]["pdhg"], j["schedule"]["iters_mean_seed"], j["schedule"]["iters_mean_warm"], j["optimal_frac"], j["iters_max"]))
for k,r in res.items(): print(k, r)
PY

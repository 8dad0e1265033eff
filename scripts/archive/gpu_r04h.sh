#!/bin/bash
# Seeded sweep: warm starts blended from the 2 / 3 nearest seeds (inverse-distance weights) vs the nearest seed alone,
# same library, same box, alternating; then the sweep GPU tests.
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
for r in 1 2; do
  for b in 1 3 2; do
    echo "== blend$b" >> $O/ab_blend.log
    timeout -k 10 300 python -u bench.py --no-cpu --no-cold-ref --steps 3 --blend $b >> $O/ab_blend.log 2>&1 || { echo "blend $b failed"; tail -20 $O/ab_blend.log; exit 1; }
  done
done
python - <<'PY'
import json, collections
v=None; res=collections.defaultdict(list)
for l in open("gpurun_out/r04h/ab_blend.log"):
    if l.startswith("=="): v=l.split()[1]
    elif l.startswith("{"):
        j=json.loads(l); res[v].append((j["value"], j["kernel_ms"]["pdhg"], j["schedule"]["iters_mean_warm"], j["optimal_frac"], j["iters_max"]))
for k,r in res.items(): print(k, r)
PY
timeout -k 10 400 python -u -m pytest tests/test_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log

#!/bin/bash
# On the GPU box: the mixed batch (scripts/mixed_batch.py) with the previous library and with the current one; the
# per-group result hashes must agree bit for bit.  Usage: scripts/ab_cascade.sh <tag> <old.so>
set -o pipefail
TAG=${1:-cascade}; OLD=$2
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 env DVH_LIB=$(pwd)/$OLD python -u scripts/mixed_batch.py $O/old.json > $O/old.log 2>&1 || { echo "old failed"; tail -20 $O/old.log; exit 1; }
timeout -k 10 300 python -u scripts/mixed_batch.py $O/new.json > $O/new.log 2>&1 || { echo "new failed"; tail -20 $O/new.log; exit 1; }
cat $O/old.json $O/new.json
python - $O/old.json $O/new.json <<'PY'
import json, sys
a, b = (json.load(open(f)) for f in sys.argv[1:3])
same = {k: a["groups"][k]["sha256"] == b["groups"][k]["sha256"] for k in a["groups"]}
print("bit-identical per group:", same, "| host syncs", a["host_syncs"], "->", b["host_syncs"], "| wall ms", a["wall_ms"], "->", b["wall_ms"])
print("paths", a["paths"], "->", b["paths"])
PY

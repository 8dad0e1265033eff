"""Summarise scripts/ab_bench.sh output: windows/s and PDHG ms per variant (mean over runs)."""
import collections
import json
import sys

v, res = None, collections.defaultdict(list)
for line in open(sys.argv[1]):
    if line.startswith("=="):
        v = line.split()[1]
    elif line.startswith("{"):
        j = json.loads(line)
        res[v].append((j["value"], j["kernel_ms"]["pdhg"], j["optimal_frac"]))
for k, r in res.items():
    print(f"{k:12s} windows/s {sum(a for a, _, _ in r) / len(r):10.1f}  pdhg ms {sum(b for _, b, _ in r) / len(r):8.2f}  "
          f"optimal {min(c for _, _, c in r)}  runs {len(r)}")

"""Turn a rocprofv3 SQ-counter pass over one bench step into profiles/pdhg_valu.json: instruction counts of the
PDHG kernel per step (summed over the step's launches), for the bench line's "compute" object.

Usage: python scripts/pmc_valu.py <pmc_dir> <windows_per_step> [out.json] [more pmc dirs ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, windows = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                              "pdhg_valu.json")
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    files = [fn for dd in [d] + sys.argv[4:] for fn in glob.glob(os.path.join(dd, "**", "*counter_collection.csv"),
                                                                  recursive=True)]
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "")
                if "pdhg_band_kernel" not in k and "pdhg_ell_kernel" not in k:
                    continue
                tot[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
                disp[fn].add(r.get("Dispatch_Id"))
    if not tot:
        raise SystemExit("no PDHG kernel counters found")
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import source_key  # noqa: E402  (the kernel sources these counters were measured on)
    nd = max(len(v) for v in disp.values())
    res = {"windows": windows, "dispatches_per_step": nd, "launches_per_step": nd,
           "source_key": source_key(),
           "counters_per_step": {c: sum(v.values()) for c, v in tot.items()},
           "note": "SQ counters summed over XCD / SE instances and over the step's PDHG launches (one pass per "
                   "counter group, each over the same single step)"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel (name prefix), every counter summed over
instances and dispatches.  Usage: python scripts/pmc_summary.py <dir> [<dir> ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def summarise(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "")[:60]
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r.get("Dispatch_Id"))
    return tot, disp


if __name__ == "__main__":
    for d in sys.argv[1:]:
        tot, disp = summarise(d)
        print(f"== {d}")
        for k in sorted(tot):
            print(f"  {k}  (dispatches {len(disp[k])})")
            for c, v in sorted(tot[k].items()):
                print(f"      {c:28s} {v:.6g}")

#!/usr/bin/env python3
"""Per-dispatch PMC summary of one kernel (name substring) from rocprofv3 csv passes, plus its average duration
from a kernel-trace pass of the same command: FP64 instruction counts / flops, VALU / LDS / SALU counts, FETCH_SIZE
(x2, the gfx950 wide-read correction of profile_round.sh) and WRITE_SIZE in bytes, achieved FP64 TFLOP/s and HBM GB/s
per dispatch.  Usage: pmc_kernel.py <kernel substring> <trace dir> <out.json> <label> <pmc dir> [pmc dir ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    pat, tdir, out, label = sys.argv[1:5]
    per = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    names = set()
    for d in sys.argv[5:]:
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as f:
                for r in csv.DictReader(f):
                    k = r.get("Kernel_Name", "")
                    if pat not in k:
                        continue
                    names.add(k[:120])
                    per[r["Counter_Name"]][(fn, r.get("Dispatch_Id"))] += float(r["Counter_Value"])
    if not per:
        raise SystemExit(f"no counters for kernels matching {pat!r}")
    avg = {c: sum(v.values()) / len(v) for c, v in per.items()}
    ndisp = {c: len(v) for c, v in per.items()}
    durs = []
    for fn in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                if pat in r.get("Kernel_Name", ""):
                    durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    res = {"label": label, "kernel_match": pat, "kernels": sorted(names), "dispatches": ndisp,
           "counters_per_dispatch": avg}
    if "FETCH_SIZE" in avg:
        res["fetch_bytes_per_dispatch"] = avg["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in avg:
        res["write_bytes_per_dispatch"] = avg["WRITE_SIZE"] * 1024
    if durs:
        # the measured (last) dispatch of the command; the first is its warm-up
        d = durs[-1]
        res["duration_s_last_dispatch"] = d
        res["durations_s"] = durs
        if "SQ_INSTS_VALU_FLOPS_FP64" in avg:
            fl = avg["SQ_INSTS_VALU_FLOPS_FP64"] * 64  # per-wave instruction flops x 64 lanes (profile_round.sh)
            res["fp64_flops_per_dispatch"] = fl
            res["fp64_tflops"] = fl / d / 1e12
            res["fp64_frac_of_78.6"] = fl / d / 1e12 / 78.64
        hb = res.get("fetch_bytes_per_dispatch", 0) + res.get("write_bytes_per_dispatch", 0)
        if hb:
            res["hbm_GBps"] = hb / d / 1e9
            res["hbm_frac_of_8000"] = hb / d / 1e9 / 8000.0
    res["note"] = ("counters averaged over the kernel's dispatches in each pass (warm-up + measured solve); SQ counters "
                   "summed over XCD / SE instances; FETCH_SIZE x2 and WRITE_SIZE x1 in KB of 1024 B")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "durations_s"}, indent=1))


if __name__ == "__main__":
    main()

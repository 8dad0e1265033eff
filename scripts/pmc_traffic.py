"""Turn rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; one counter per pass) into profiles/pdhg_traffic.json.

Usage: python scripts/pmc_traffic.py <fetch_dir> <write_dir> <windows_per_step> [out.json] [launches_per_step]

With the seeded sweep schedule (bench.py default) one step is two launches of the PDHG kernel (seed phase, warm
phase); hbm_bytes_per_step sums them (the PMC runs do exactly one step and skip the cold reference solves).

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters).  Per MI355X_MICROARCH.md section HBM: on
gfx950 FETCH_SIZE reports half of the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is taken
as is.  Both include Infinity-Cache hits (memory-side L2 requests), so they are an upper bound on HBM bytes.
The dominant kernel is the PDHG kernel (pdhg_band_kernel<...> for battery-banded windows, else
pdhg_ell_kernel<...>); values are averaged over its dispatches.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def read_counter(d, name):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(float)  # (dispatch id, kernel) -> summed value over XCD/SE instances
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != name:
                    continue
                key = (r.get("Dispatch_Id"), r.get("Kernel_Name", ""))
                per[key] += float(r["Counter_Value"])
    by_kernel = defaultdict(list)
    for (_, k), v in per.items():
        by_kernel[k].append(v)
    return by_kernel


def main():
    fdir, wdir, windows = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                              "pdhg_traffic.json")
    lps = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    fetch = read_counter(fdir, "FETCH_SIZE")
    write = read_counter(wdir, "WRITE_SIZE")
    kern = [k for k in fetch if "pdhg_band_kernel" in k] or [k for k in fetch if "pdhg_ell_kernel" in k]
    if not kern:
        raise SystemExit(f"no PDHG kernel in {list(fetch)}")
    fv = [v for k in kern for v in fetch[k]]
    wv = [v for k in kern for v in write.get(k, [])]
    f_kb = sum(fv) / len(fv)
    w_kb = sum(wv) / len(wv) if wv else 0.0
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import source_key  # noqa: E402
    res = {
        "source_key": source_key(),
        "kernel": re.search(r"pdhg_(band|ell)_kernel<[^>]*>", kern[0]).group(0),
        "windows": windows,
        "dispatches_fetch": len(fv), "dispatches_write": len(wv),
        "fetch_size_kb_raw": f_kb, "write_size_kb": w_kb,
        "hbm_bytes_per_launch": 2.0 * f_kb * 1024.0 + w_kb * 1024.0,
        "launches_per_step": lps,
        "hbm_bytes_per_step": (2.0 * f_kb * 1024.0 + w_kb * 1024.0) * lps,
        "correction": "FETCH_SIZE x2 (gfx950 wide-read under-count), WRITE_SIZE x1; KB = 1024 B",
        "other_kernels": {re.sub(r"^void |\(.*$", "", k)[:80]: {"fetch_kb": sum(v) / len(v)} for k, v in fetch.items()
                          if k not in kern},
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where a kernel's spills sit: scratch loads / stores of each kernel in a HIP source, counted by the loop depth LLVM
annotates on their basic block (gfx950 ISA from hipcc -S with the library's per-source flags).  For the persistent band
forms depth 1 is the loop over windows (per-window set-up and write-back), depth 2 the iteration loop; a scratch op at
depth 2 may still sit in a rarely taken branch (check iterations, restarts, the Halpern-table reload every 64
iterations) -- the listing with --lines shows each one's block.

Usage: python scripts/spill_sites.py [file.hip ...] [--lines]   (default: dvh_band_persist.hip dvh_band_persist_ice.hip dvh_kernels.hip)
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "der-vet_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))
from dervet_hip.build import EXTRA_FLAGS  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from spills import short  # noqa: E402


def isa(path):
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-S", "--offload-device-only",
           "-Wno-unused-result", "-Wno-unused-value", *EXTRA_FLAGS.get(os.path.basename(path), ()), path, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-4000:])
    with open(out) as f:
        return f.read().split("\n")


def sites(lines):
    fns = [(i, re.search(r"\.type\s+(\S+),@function", ln).group(1)) for i, ln in enumerate(lines) if "@function" in ln]
    for k, (s0, name) in enumerate(fns):
        body = lines[s0:fns[k + 1][0] if k + 1 < len(fns) else len(lines)]
        depth, blk, found = 0, "", []
        for ln in body:
            if re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", ln):
                m = re.search(r"Depth=(\d+)", ln)
                depth, blk = (int(m.group(1)) if m else 0), ln.split(":")[0]
            if "scratch_" in ln:
                found.append((depth, blk, ln.strip()))
        yield name, found


def main(argv):
    show = "--lines" in argv
    files = [a for a in argv if not a.startswith("--")] or ["dvh_band_persist.hip", "dvh_band_persist_ice.hip", "dvh_kernels.hip"]
    for f in files:
        p = f if os.path.exists(f) else os.path.join(CSRC, f)
        for name, found in sites(isa(p)):
            if not found:
                continue
            c = Counter(d for d, _, _ in found)
            print(f"{os.path.basename(p):22s} {short(name):45s} scratch ops {len(found):4d}  by loop depth "
                  + " ".join(f"{d}:{c[d]}" for d in sorted(c)))
            if show:
                for d, b, ln in found:
                    print(f"    depth {d} {b:14s} {ln}")


if __name__ == "__main__":
    main(sys.argv[1:])

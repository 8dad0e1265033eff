"""Per-kernel VGPR / spill counts of the HIP sources (hipcc -Rpass-analysis=kernel-resource-usage, gfx950).

Usage: python scripts/spills.py [file.hip ...]   (default: every source of libdervet_hip.so)
Prints one line per kernel: VGPRs, spilled VGPRs, spilled SGPRs, occupancy (waves per SIMD), name.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "der-vet_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))
from dervet_hip.build import EXTRA_FLAGS  # noqa: E402  (per-source flags of the library build)
DEFAULT = ["dvh_band.hip", "dvh_band_persist.hip", "dvh_band_persist_ice.hip", "dvh_kernels.hip", "dvh_chain.hip", "dvh_large.hip", "dvh_build.hip", "dvh_sweep.hip",
           "dvh_outage.hip"]


def usage(path, extra=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "--offload-device-only",
           "-Rpass-analysis=kernel-resource-usage", "-Wno-unused-result", "-Wno-unused-value", *extra, path,
           "-o", os.devnull]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-4000:])
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            out.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    return out


def short(name):
    m = re.search(r"_GLOBAL__N_1\d+(\w+?)I(.*)EEvNS", name)
    if not m:
        return name
    args = re.findall(r"L([ib])(\d+)E", m.group(2))
    return m.group(1) + "<" + ",".join(v for _, v in args) + ">"


def main(argv):
    files = argv or DEFAULT
    for f in files:
        p = f if os.path.exists(f) else os.path.join(CSRC, f)
        for k in usage(p, EXTRA_FLAGS.get(os.path.basename(p), ())):
            if "VGPRs" not in k:
                continue
            print(f"{os.path.basename(p):16s} vgpr {k['VGPRs']:>4s} spill_v {k.get('VGPRs Spill', '?'):>3s} "
                  f"spill_s {k.get('SGPRs Spill', '?'):>3s} occ {k.get('Occupancy [waves/SIMD]', '?'):>2s}  "
                  f"{short(k['name'])}")


if __name__ == "__main__":
    main(sys.argv[1:])

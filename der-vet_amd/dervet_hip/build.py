"""Build libdervet_hip.so in-tree for gfx950 (hipcc cross-compiles; no GPU needed).

Usage: python -m dervet_hip.build   (or dervet_hip.build.build())
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "csrc")
LIB = os.path.join(HERE, "libdervet_hip.so")
SOURCES = ["dvh_kernels.hip", "dvh_band.hip", "dvh_chain.hip", "dvh_build.hip", "dvh_sweep.hip", "dvh_large.hip", "dvh_outage.hip", "dvh_api.cpp"]
HEADERS = ["dvh_internal.h", "dvh_device.h", os.path.join("..", "..", "include", "dervet_hip.h")]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def build(force=False, verbose=False):
    if not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-result", "-Wno-unused-value", "-o", LIB + ".tmp"] + [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc failed building libdervet_hip.so")
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))

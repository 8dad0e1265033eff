"""Build libdervet_hip.so in-tree for gfx950 (hipcc cross-compiles; no GPU needed).

Usage: python -m dervet_hip.build   (or dervet_hip.build.build())
"""
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "csrc")
LIB = os.path.join(HERE, "libdervet_hip.so")
# the build configuration the library was linked with (flags and compiler string), written by build(): bench.py keys
# its PMC profiles to it without running hipcc from a process that may already hold the GPU (under rocprofv3 --pmc it
# does, and the GPU box refuses an exec from such a process)
BUILDINFO = os.path.join(HERE, "libdervet_hip.buildinfo.json")
SOURCES = ["dvh_kernels.hip", "dvh_band.hip", "dvh_band_persist.hip", "dvh_band_persist_ice.hip", "dvh_chain.hip", "dvh_build.hip", "dvh_sweep.hip", "dvh_series.hip", "dvh_route.hip", "dvh_large.hip", "dvh_outage.hip",
           "dvh_api.cpp", "dvh_validate.cpp", "dvh_comm.cpp"]
# per-source flags: the band kernel's persistent forms without machine-level loop-invariant code motion (their loop
# invariants, hoisted out of the loop over windows, spilled; csrc/dvh_band_persist.hip), the battery form with the
# AMDGPU scheduler's register-pressure trackers (+2.1 % on the bench; the ICE form is slower with them)
EXTRA_FLAGS = {"dvh_band_persist.hip": ["-mllvm", "-disable-machine-licm", "-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
               "dvh_band_persist_ice.hip": ["-mllvm", "-disable-machine-licm"],
               # the team kernel (config 3 DCM + PV 162 -> 151 ms) and the ELL / generic kernels (1,095 market days
               # 5.35 -> 5.12 ms) without machine LICM too: profiles/r05zj_chain_kernels_flags.log
               "dvh_chain.hip": ["-mllvm", "-disable-machine-licm"],
               "dvh_kernels.hip": ["-mllvm", "-disable-machine-licm"]}
INCLUDES = {"dvh_band_persist.hip": "dvh_band.hip",  # (a one-line source around another: its compile time)
            "dvh_band_persist_ice.hip": "dvh_band.hip"}
# flags of every object (build() and build_variant()); bench.source_key() hashes them with EXTRA_FLAGS and the compiler
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result", "-Wno-unused-value"]
HEADERS = ["dvh_internal.h", "dvh_device.h", "dvh_validate.h", "dvh_rng.h", "dvh_ziggurat.h", os.path.join("..", "..", "include", "dervet_hip.h")]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    # this file too: its per-source flags change the objects
    return os.path.getmtime(os.path.abspath(__file__)) > t or \
        any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def build(force=False, verbose=False):
    """Compile every source to an object in parallel (the ELL / band instantiations make dvh_kernels.hip the long
    pole, ~2 min), then link.  Each kernel is launched from its own translation unit, so no -fgpu-rdc."""
    if not force and not _stale():
        if not os.path.exists(BUILDINFO):
            _write_buildinfo()
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = list(FLAGS)
    objdir = os.path.join(HERE, "build_obj")
    os.makedirs(objdir, exist_ok=True)
    # longest first, so the pool's tail is short
    order = sorted(SOURCES, key=lambda f: -os.path.getsize(os.path.join(CSRC, INCLUDES.get(f, f))))
    objs = {f: os.path.join(objdir, f + ".o") for f in SOURCES}

    def compile_one(f):
        cmd = [hipcc, *flags, *EXTRA_FLAGS.get(f, []), "-c", os.path.join(CSRC, f), "-o", objs[f]]
        if verbose:
            print(" ".join(cmd), flush=True)
        return f, subprocess.run(cmd, capture_output=True, text=True)

    jobs = int(os.environ.get("DVH_BUILD_JOBS", min(len(SOURCES), os.cpu_count() or 1, 16)))
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        results = list(ex.map(compile_one, order))
    failed = [(f, r) for f, r in results if r.returncode != 0]
    for f, r in failed:
        sys.stderr.write(f"--- {f}\n" + r.stdout + r.stderr)
    if failed:
        raise RuntimeError("hipcc failed building libdervet_hip.so: " + ", ".join(f for f, _ in failed))
    cmd = [hipcc, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", LIB + ".tmp"] + [objs[f] for f in SOURCES]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc failed linking libdervet_hip.so")
    os.replace(LIB + ".tmp", LIB)
    _write_buildinfo()
    return LIB


def _write_buildinfo():
    cfg = _current_config(compiler_version())
    with open(BUILDINFO + ".tmp", "w") as f:
        json.dump(cfg, f, sort_keys=True)
    os.replace(BUILDINFO + ".tmp", BUILDINFO)


def build_variant(out, defines, recompile=("dvh_band.hip", "dvh_band_persist.hip", "dvh_band_persist_ice.hip"),
                  verbose=False):
    """A/B helper: the library with ``defines`` (e.g. ["-DDVH_BAND_PROBE=1"]) applied to the sources in
    ``recompile`` (their objects go to build_obj/<name>/), every other object taken from the default build."""
    build()
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = [*FLAGS, *defines]
    name = os.path.splitext(os.path.basename(out))[0]
    objdir = os.path.join(HERE, "build_obj", name)
    os.makedirs(objdir, exist_ok=True)
    objs = {f: os.path.join(HERE, "build_obj", f + ".o") for f in SOURCES}

    def compile_one(f):
        objs[f] = os.path.join(objdir, f + ".o")
        cmd = [hipcc, *flags, *EXTRA_FLAGS.get(f, []), "-c", os.path.join(CSRC, f), "-o", objs[f]]
        if verbose:
            print(" ".join(cmd), flush=True)
        return f, subprocess.run(cmd, capture_output=True, text=True)

    with ThreadPoolExecutor(max_workers=max(1, len(recompile))) as ex:
        results = list(ex.map(compile_one, recompile))
    failed = [(f, r) for f, r in results if r.returncode != 0]
    for f, r in failed:
        sys.stderr.write(f"--- {f}\n" + r.stdout + r.stderr)
    if failed:
        raise RuntimeError("hipcc failed building variant " + name)
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    cmd = [hipcc, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out] + [objs[f] for f in SOURCES]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc failed linking variant " + name)
    return out


def compiler_version():
    """The hipcc / clang version string the objects are built with ("unknown" if hipcc cannot be run)."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    try:
        r = subprocess.run([hipcc, "--version"], capture_output=True, text=True, timeout=60)
        lines = [ln.strip() for ln in r.stdout.splitlines() if ln.strip()]
        # HIP version + the clang line (drop the install-dir lines, which differ between boxes of one image)
        return " | ".join(ln for ln in lines if not ln.startswith("InstalledDir")) or "unknown"
    except (OSError, subprocess.SubprocessError):
        return "unknown"


def _current_config(compiler):
    return {"flags": FLAGS, "extra_flags": {k: EXTRA_FLAGS[k] for k in sorted(EXTRA_FLAGS)}, "compiler": compiler}


def build_config():
    """Everything besides the sources that decides the machine code: common and per-source flags, compiler.  The
    compiler string is the one build() recorded with the library when its flags are the current ones; hipcc is asked
    only when there is no such record."""
    try:
        with open(BUILDINFO) as f:
            rec = json.load(f)
        if rec == _current_config(rec.get("compiler")) and rec.get("compiler"):
            return rec
    except (OSError, ValueError):
        pass
    return _current_config(compiler_version())


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))

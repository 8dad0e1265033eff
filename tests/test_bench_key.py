"""bench.py's PMC key: the committed PMC JSONs under profiles/ feed the roofline only while
they were measured on the same machine code -- the kernel sources AND the build configuration (common flags,
per-source flags such as -disable-machine-licm, the compiler version)."""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from dervet_hip import build  # noqa: E402


def _key(cfg):
    return bench.source_key(json.dumps(cfg, sort_keys=True))


def test_flag_only_change_changes_the_key():
    cfg = build.build_config()
    base = _key(cfg)
    assert base == bench.source_key()
    flipped = copy.deepcopy(cfg)
    flipped["extra_flags"]["dvh_band_persist.hip"] = [f for f in flipped["extra_flags"]["dvh_band_persist.hip"]
                                                      if "trackers" not in f]
    assert _key(flipped) != base
    opt = copy.deepcopy(cfg)
    opt["flags"] = [f if f != "-O3" else "-O2" for f in opt["flags"]]
    assert _key(opt) != base
    comp = copy.deepcopy(cfg)
    comp["compiler"] = comp["compiler"] + " (other)"
    assert _key(comp) != base


def test_committed_pmc_profiles_carry_the_current_key():
    """The PMC JSONs the bench line reads were measured on the current sources and build configuration."""
    key = bench.source_key()
    for name in ("pdhg_traffic", "pdhg_valu"):
        with open(os.path.join(ROOT, "profiles", name + ".json")) as f:
            assert json.load(f)["source_key"] == key, name


def test_build_config_reads_the_recorded_compiler_and_ignores_a_stale_record(tmp_path, monkeypatch):
    """build() records the build configuration with the library; build_config() uses the recorded compiler string only
    while the recorded flags are the current ones (so bench.py forms its key without running hipcc from a process that
    may hold the GPU), and asks hipcc otherwise."""
    rec = tmp_path / "buildinfo.json"
    monkeypatch.setattr(build, "BUILDINFO", str(rec))
    monkeypatch.setattr(build, "compiler_version", lambda: "hipcc (asked)")
    cur = {"flags": build.FLAGS, "extra_flags": {k: build.EXTRA_FLAGS[k] for k in sorted(build.EXTRA_FLAGS)},
           "compiler": "hipcc (recorded)"}
    rec.write_text(json.dumps(cur))
    assert build.build_config()["compiler"] == "hipcc (recorded)"
    stale = dict(cur, flags=cur["flags"] + ["-DSTALE"])
    rec.write_text(json.dumps(stale))
    assert build.build_config()["compiler"] == "hipcc (asked)"
    rec.unlink()
    assert build.build_config()["compiler"] == "hipcc (asked)"

#!/usr/bin/env python3
"""Generates der-vet_amd/csrc/dvh_ziggurat.h: the 256-strip ziggurat tables numpy's Generator.standard_normal
uses (numpy/random/src/distributions/ziggurat_constants.h: ki_double, wi_double, fi_double), recovered from numpy's
own output so that the device generator (csrc/dvh_rng.h) draws bit-identical normals.

numpy ships the tables only inside its compiled extension, so they are recovered, not copied:
  * the PCG64 + SeedSequence stream is restated (pcg64_stream below; checked against PCG64.random_raw);
  * 1,000,000 standard normals are drawn one at a time while the bit generator's state is tracked, which gives for
    every draw the raw words it consumed; a draw that consumed one word took the fast path, x = rabs * wi[idx],
    so wi[idx] is the one double w with fl(rabs * w) == |x| for every such draw (unique for all 256 strips;
    strip 1 has no fast path and is recovered from first-wedge accepts);
  * x_i = wi[i] * 2^52 are the strip edges (x_255 = r = ziggurat_nor_r; wi[0] is the base strip's v / f(r));
    ki[i] = floor(2^52 x_{i-1} / x_i) (ki[0] = floor(2^52 r / (v / f(r))), ki[1] = 0: the top strip always takes
    the wedge test) -- every value lies inside the interval the draws bound it to -- and fi[i] = exp(-x_i^2 / 2)
    (fi[0] = 1), which reproduces every wedge decision;
  * the complete restated draw (fast path, wedge, tail via log1p) is checked bit for bit against numpy's
    lognormal / standard_normal / uniform sequence of 200 config-4 scenarios.
Usage: python scripts/gen_ziggurat_tables.py  (about 15 s; rewrites the header only if every check passes)."""
import math
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "der-vet_amd", "csrc", "dvh_ziggurat.h")
M32, M64, M128 = 0xFFFFFFFF, (1 << 64) - 1, (1 << 128) - 1
PCG_MULT = (2549297995355413924 << 64) | 4865540595714422341
R = 3.6541528853610087963519472518        # ziggurat_nor_r
RINV = 0.27366123732975827203338247596    # ziggurat_nor_inv_r


def seed_state(seed):
    """SeedSequence(seed).generate_state(4, uint64) -> PCG64 (state, inc) after pcg64_set_seed."""
    ent = []
    n = seed
    while True:
        ent.append(n & M32)
        n >>= 32
        if n == 0:
            break
    hc = 0x43b0d7e5

    def hashmix(v):
        nonlocal hc
        v = (v ^ hc) & M32
        hc = (hc * 0x931e8875) & M32
        v = (v * hc) & M32
        return v ^ (v >> 16)

    def mix(x, y):
        r = (0xca01f9dd * x - 0x4973f715 * y) & M32
        return r ^ (r >> 16)

    pool = [hashmix(ent[i]) if i < len(ent) else hashmix(0) for i in range(4)]
    for s in range(4):
        for d in range(4):
            if s != d:
                pool[d] = mix(pool[d], hashmix(pool[s]))
    for s in range(4, len(ent)):
        for d in range(4):
            pool[d] = mix(pool[d], hashmix(ent[s]))
    hb, w = 0x8b51f9dd, []
    for i in range(8):
        v = (pool[i % 4] ^ hb) & M32
        hb = (hb * 0x58f38ded) & M32
        v = (v * hb) & M32
        w.append(v ^ (v >> 16))
    u64 = [w[2 * i] | (w[2 * i + 1] << 32) for i in range(4)]
    inc = ((((u64[2] << 64) | u64[3]) << 1) | 1) & M128
    st = inc                                            # state 0 stepped once
    st = (st + ((u64[0] << 64) | u64[1])) & M128
    return (st * PCG_MULT + inc) & M128, inc


class Pcg64:
    def __init__(self, seed):
        self.st, self.inc = seed_state(seed)

    def next(self):
        self.st = (self.st * PCG_MULT + self.inc) & M128
        s = self.st
        x = ((s >> 64) ^ s) & M64
        rot = s >> 122
        return ((x >> rot) | (x << ((64 - rot) & 63))) & M64

    def next_double(self):
        return (self.next() >> 11) * (1.0 / 9007199254740992.0)


def check_stream():
    for seed in (0, 1, 20250217, 20250217 + 9999, 2 ** 40 + 5):
        g = Pcg64(seed)
        assert [g.next() for _ in range(8)] == np.random.PCG64(seed).random_raw(8).tolist(), seed


def sample(n, seed=7):
    """(idx, rabs, words consumed, |x|, raw words) of n numpy standard normals."""
    rng = np.random.Generator(np.random.PCG64(seed))
    bg, g, out = rng.bit_generator, Pcg64(seed), []
    for _ in range(n):
        z = rng.standard_normal()
        target, raws = bg.state["state"]["state"], []
        while g.st != target:
            raws.append(g.next())
            assert len(raws) < 64
        r = raws[0]
        out.append((r & 0xff, ((r >> 8) >> 1) & 0x000fffffffffffff, len(raws), abs(z), raws))
    return out


def exact_w(pairs):
    """The double w with fl(rabs * w) == x for all (rabs, x)."""
    cand = None
    for rabs, x in pairs[:64]:
        w = x / rabs
        for _ in range(4):
            w = float(np.nextafter(w, -np.inf))
        cs = set()
        for _ in range(9):
            if float(np.float64(rabs) * np.float64(w)) == x:
                cs.add(w)
            w = float(np.nextafter(w, np.inf))
        cand = cs if cand is None else cand & cs
    ok = [w for w in sorted(cand or ()) if all(float(np.float64(r) * np.float64(w)) == x for r, x in pairs)]
    if len(ok) != 1:
        raise SystemExit(f"wi not pinned: {len(ok)} candidates")
    return ok[0]


def recover(n=1_000_000):
    S = sample(n)
    wi = []
    for idx in range(256):
        fast = [(rabs, x) for i, rabs, c, x, _ in S if i == idx and c == (1 if idx != 1 else 2)]
        wi.append(exact_w(fast))
    X = [w * 2.0 ** 52 for w in wi]
    assert X[255] == R
    ki = [int(math.floor(R / X[0] * 2.0 ** 52)), 0] + [int(math.floor(X[i - 1] / X[i] * 2.0 ** 52))
                                                       for i in range(2, 256)]
    fi = [1.0] + [math.exp(-0.5 * X[i] * X[i]) for i in range(1, 256)]
    for idx in range(2, 256):       # ki inside the interval the draws bound it to
        lo = max((rabs for i, rabs, c, _, _ in S if i == idx and c == 1), default=-1)
        hi = min((rabs for i, rabs, c, _, _ in S if i == idx and c > 1), default=1 << 52)
        assert lo < ki[idx] <= hi, idx
    for idx, rabs, c, x, raws in S:  # every first wedge decision
        if c >= 2 and idx != 0:
            xx = rabs * wi[idx]
            lhs = (fi[idx - 1] - fi[idx]) * ((raws[1] >> 11) * (1.0 / 9007199254740992.0)) + fi[idx]
            assert (lhs < math.exp(-0.5 * xx * xx)) == (c == 2)
    return wi, ki, fi


def normal(g, wi, ki, fi):
    """Restated random_standard_normal (numpy distributions.c) on the restated stream."""
    while True:
        r = g.next()
        idx = r & 0xff
        r >>= 8
        sign, rabs = r & 1, (r >> 1) & 0x000fffffffffffff
        x = rabs * wi[idx]
        if sign:
            x = -x
        if rabs < ki[idx]:
            return x
        if idx == 0:
            while True:
                xx = -RINV * math.log1p(-g.next_double())
                yy = -math.log1p(-g.next_double())
                if yy + yy > xx * xx:
                    return -(R + xx) if (rabs >> 8) & 1 else R + xx
        elif (fi[idx - 1] - fi[idx]) * g.next_double() + fi[idx] < math.exp(-0.5 * x * x):
            return x


def check_sequences(wi, ki, fi, scenarios=200, seed0=20250217):
    for s in range(scenarios):
        rng = np.random.Generator(np.random.PCG64(seed0 + s))
        ref = np.concatenate([[rng.lognormal(0.0, 0.15)], rng.standard_normal(8760), [rng.uniform(0.7, 1.3)]])
        g = Pcg64(seed0 + s)
        z0 = normal(g, wi, ki, fi)
        mine = [math.exp(0.0 + 0.15 * z0)] + [normal(g, wi, ki, fi) for _ in range(8760)]
        mine.append(0.7 + (1.3 - 0.7) * g.next_double())
        assert np.array_equal(np.array(mine), ref), s


def write(wi, ki, fi):
    h = lambda d: "0x%016xULL" % struct.unpack("<Q", struct.pack("<d", float(d)))[0]
    rows = lambda vals: ",\n".join("    " + ", ".join(vals[i:i + 4]) for i in range(0, 256, 4))
    with open(OUT, "w") as f:
        f.write("// Generated by scripts/gen_ziggurat_tables.py -- do not edit.\n"
                "// numpy Generator.standard_normal's 256-strip ziggurat (distributions.c random_standard_normal):\n"
                "// wi = strip edge / 2^52 (bits of the double), ki = fast-path bound on the 52-bit mantissa draw,\n"
                "// fi = exp(-x^2 / 2) at the edge (bits).  Recovered from and checked against numpy's output.\n"
                "#pragma once\n#include <cstdint>\n\nnamespace dvh {\nnamespace zig {\n")
        f.write("static constexpr uint64_t kWiBits[256] = {\n" + rows([h(w) for w in wi]) + "};\n")
        f.write("static constexpr uint64_t kKi[256] = {\n" + rows(["0x%013xULL" % k for k in ki]) + "};\n")
        f.write("static constexpr uint64_t kFiBits[256] = {\n" + rows([h(v) for v in fi]) + "};\n")
        f.write("}  // namespace zig\n}  // namespace dvh\n")


def main():
    check_stream()
    wi, ki, fi = recover()
    check_sequences(wi, ki, fi)
    write(wi, ki, fi)
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())

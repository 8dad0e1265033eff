// numpy-identical random draws for the synthetic scenario generator (BASELINE config 4 / 5):
// SeedSequence -> PCG64 (XSL-RR 128/64) -> Generator.standard_normal (256-strip ziggurat) / uniform, restated so
// that a device thread per scenario draws exactly the numbers `np.random.Generator(np.random.PCG64(seed))` draws
// on the host (dervet_hip/lp/scenarios.py sweep_parameters; tests/test_series.py checks the host build of this
// header against numpy, tests/test_gpu_series.py the device build).
//
// Every floating-point operation is written out one IEEE operation at a time and the translation units that use
// this header are compiled with -ffp-contract=off (an FMA would round differently).  The ziggurat's tail uses
// log1p: `log1p_fdlibm` restates the fdlibm algorithm glibc's libm implements (s_log1p.c), checked bit for bit
// against the host libm on the generator's whole input domain (tests/test_series.py).  The wedge test compares
// against exp(-x^2/2): its outcome, not its value, matters; a device exp within an ulp gives the same decision
// unless the two sides are within a few ulps, which `normal` reports (the draw is then not trusted).
//
// Included by g++ (tests) and hipcc (device), hence DVH_HD.
#pragma once
#include <cstdint>
#include <cstring>

#include "dvh_ziggurat.h"

#if defined(__HIPCC__)
#define DVH_HD __host__ __device__
#else
#define DVH_HD
#endif

namespace dvh {
namespace rng {

typedef unsigned __int128 u128;

DVH_HD inline double bits_to_double(uint64_t b) {
  double d;
  memcpy(&d, &b, sizeof d);
  return d;
}
DVH_HD inline uint64_t double_to_bits(double d) {
  uint64_t b;
  memcpy(&b, &d, sizeof b);
  return b;
}

// ---- numpy SeedSequence(entropy).generate_state(4, uint64) (bit_generator.pyx) + pcg64_set_seed.
struct Pcg64 {
  u128 state, inc;
};

DVH_HD inline uint32_t ss_hashmix(uint32_t v, uint32_t& hc) {
  v ^= hc;
  hc *= 0x931e8875u;
  v *= hc;
  v ^= v >> 16;
  return v;
}
DVH_HD inline uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
  r ^= r >> 16;
  return r;
}

// entropy: a non-negative integer below 2^64 (numpy splits it into little-endian 32-bit words, at least one)
DVH_HD inline Pcg64 seed_pcg64(uint64_t entropy) {
  uint32_t ent[2] = {(uint32_t)entropy, (uint32_t)(entropy >> 32)};
  const int n_ent = (entropy >> 32) ? 2 : 1;
  uint32_t pool[4];
  uint32_t hc = 0x43b0d7e5u;
  for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i < n_ent ? ent[i] : 0u, hc);
  for (int s = 0; s < 4; ++s)
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
  uint32_t w[8];
  uint32_t hb = 0x8b51f9ddu;
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i & 3] ^ hb;
    hb *= 0x58f38dedu;
    v *= hb;
    v ^= v >> 16;
    w[i] = v;
  }
  uint64_t u[4];
  for (int i = 0; i < 4; ++i) u[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  const u128 mult = ((u128)2549297995355413924ULL << 64) | (u128)4865540595714422341ULL;
  const u128 initstate = ((u128)u[0] << 64) | (u128)u[1];
  const u128 initseq = ((u128)u[2] << 64) | (u128)u[3];
  Pcg64 g;
  g.inc = (initseq << 1) | (u128)1;
  g.state = g.inc;                     // state 0 stepped once: 0 * mult + inc
  g.state += initstate;
  g.state = g.state * mult + g.inc;
  return g;
}

DVH_HD inline uint64_t next_u64(Pcg64& g) {
  const u128 mult = ((u128)2549297995355413924ULL << 64) | (u128)4865540595714422341ULL;
  g.state = g.state * mult + g.inc;
  const uint64_t x = (uint64_t)(g.state >> 64) ^ (uint64_t)g.state;
  const unsigned rot = (unsigned)(g.state >> 122);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

DVH_HD inline double next_double(Pcg64& g) {
  return (double)(next_u64(g) >> 11) * (1.0 / 9007199254740992.0);
}

// ---- log1p as glibc's libm computes it (fdlibm s_log1p.c; the polynomial in glibc's split form).
DVH_HD inline double log1p_fdlibm(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01, Lp3 = 2.857142874366239149e-01,
               Lp4 = 2.222219843214978396e-01, Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
               Lp7 = 1.479819860511658591e-01;
  const uint64_t bx = double_to_bits(x);
  const int32_t hx = (int32_t)(bx >> 32);
  const int32_t ax = hx & 0x7fffffff;
  int32_t k = 1, hu = 0;
  double f = 0.0, c = 0.0;
  if (hx < 0x3FDA827A) {                      // x < 0.41422
    if (ax >= 0x3ff00000) {                   // x <= -1
      if (x == -1.0) return -__builtin_inf();
      return __builtin_nan("");
    }
    if (ax < 0x3e200000) {                    // |x| < 2^-29
      if (ax < 0x3c900000) return x;          // |x| < 2^-54
      return x - x * x * 0.5;
    }
    if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {  // -0.2929 < x < 0.41422 (fdlibm's bound, as glibc 2.35)
      k = 0;
      f = x;
      hu = 1;
    }
  } else if (hx >= 0x7ff00000) {
    return x + x;
  }
  if (k != 0) {
    double u;
    if (hx < 0x43400000) {
      u = 1.0 + x;
      hu = (int32_t)(double_to_bits(u) >> 32);
      k = (hu >> 20) - 1023;
      c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
      c /= u;
    } else {
      u = x;
      hu = (int32_t)(double_to_bits(u) >> 32);
      k = (hu >> 20) - 1023;
      c = 0;
    }
    hu &= 0x000fffff;
    uint64_t bu = double_to_bits(u) & 0xffffffffULL;
    if (hu < 0x6a09e) {
      bu |= (uint64_t)(uint32_t)(hu | 0x3ff00000) << 32;     // normalise u
    } else {
      k += 1;
      bu |= (uint64_t)(uint32_t)(hu | 0x3fe00000) << 32;     // normalise u / 2
      hu = (0x00100000 - hu) >> 2;
    }
    f = bits_to_double(bu) - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  if (hu == 0) {                               // |f| < 2^-20
    if (f == 0.0) {
      if (k == 0) return 0.0;
      c += k * ln2_lo;
      return k * ln2_hi + c;
    }
    const double R = hfsq * (1.0 - 0.66666666666666666 * f);
    if (k == 0) return f - R;
    return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double R1 = z * Lp1, z2 = z * z;
  const double R2 = Lp2 + z * Lp3, z4 = z2 * z2;
  const double R3 = Lp4 + z * Lp5, z6 = z4 * z2;
  const double R4 = Lp6 + z * Lp7;
  const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

// ---- Generator.standard_normal (numpy distributions.c random_standard_normal).  `Exp` evaluates exp(-x^2/2) for
// the wedge test; `ambiguous` is raised when that test's two sides are within 2^-40 relative (the decision could
// depend on the last bits of exp).
template <class Exp>
DVH_HD inline double normal(Pcg64& g, Exp exp_fn, int& ambiguous) {
  const double r = 3.6541528853610087963519472518, rinv = 0.27366123732975827203338247596;
  for (;;) {
    uint64_t u = next_u64(g);
    const int idx = (int)(u & 0xff);
    u >>= 8;
    const int sign = (int)(u & 1);
    const uint64_t rabs = (u >> 1) & 0x000fffffffffffffULL;
    double x = (double)rabs * bits_to_double(zig::kWiBits[idx]);
    if (sign) x = -x;
    if (rabs < zig::kKi[idx]) return x;
    if (idx == 0) {
      for (;;) {
        const double xx = -rinv * log1p_fdlibm(-next_double(g));
        const double yy = -log1p_fdlibm(-next_double(g));
        if (yy + yy > xx * xx) return ((rabs >> 8) & 1) ? -(r + xx) : r + xx;
      }
    }
    const double fhi = bits_to_double(zig::kFiBits[idx - 1]), flo = bits_to_double(zig::kFiBits[idx]);
    const double lhs = (fhi - flo) * next_double(g) + flo;
    const double rhs = exp_fn(-0.5 * x * x);
    const double gap = lhs - rhs;
    if ((gap < 0 ? -gap : gap) <= rhs * 0x1p-40) ambiguous = 1;
    if (lhs < rhs) return x;
  }
}

}  // namespace rng
}  // namespace dvh

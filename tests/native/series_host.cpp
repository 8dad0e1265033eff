// Host build of der-vet_amd/csrc/dvh_rng.h for tests/test_series.py (g++ -O2 -ffp-contract=off): the device
// generator's arithmetic checked against numpy / the host libm without a GPU.  Test code, not shipped.
#include <cmath>
#include <cstdint>

#include "dvh_rng.h"

namespace {
struct HostExp {
  double operator()(double v) const { return std::exp(v); }
};
uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
}  // namespace

extern "C" {
// The series_draws_kernel's per-scenario loop (dvh_series.hip), one scenario after the other.
int series_draws_host(const uint64_t* seeds, int count, int steps, int n_unif, double a1, double innov, double* z0,
                      double* ar, double* unif) {
  int amb = 0;
  const HostExp ex;
  for (int i = 0; i < count; ++i) {
    dvh::rng::Pcg64 g = dvh::rng::seed_pcg64(seeds[i]);
    z0[i] = dvh::rng::normal(g, ex, amb);
    double z = 0.0;
    for (int t = 0; t < steps; ++t) {
      const double e = dvh::rng::normal(g, ex, amb);
      const double x = t == 0 ? e : e * innov;
      const double y = z + x;
      z = x * 0.0 - y * a1;
      ar[(int64_t)i * steps + t] = y;
    }
    for (int k = 0; k < n_unif; ++k) unif[(int64_t)i * n_unif + k] = dvh::rng::next_double(g);
  }
  return amb;
}

void raw_words(uint64_t seed, int n, uint64_t* out) {
  dvh::rng::Pcg64 g = dvh::rng::seed_pcg64(seed);
  for (int i = 0; i < n; ++i) out[i] = dvh::rng::next_u64(g);
}

// log1p_fdlibm vs the host libm: n random next_double words u (log1p(-u): the ziggurat tail's arguments) plus n
// arguments uniform in (-1, 1), and a dense sweep of `sweep` doubles around each branch boundary.  Returns mismatches.
long long log1p_mismatches(long long n, long long sweep) {
  uint64_t s = 12345;
  long long bad = 0;
  auto check = [&](double x) {
    if (dvh::rng::double_to_bits(dvh::rng::log1p_fdlibm(x)) != dvh::rng::double_to_bits(std::log1p(x))) ++bad;
  };
  for (long long i = 0; i < n; ++i) {
    check(-((double)(splitmix(s) >> 11) * (1.0 / 9007199254740992.0)));
    check(((double)(splitmix(s) >> 11) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0);
  }
  const double starts[] = {-0.2928932188134524, -0.41, -1.0 + 1e-9, -1e-5, -9.5367431640625e-07, -0.5,
                           -0.70710678118654746, 0.41421356237309503, 1.8626451492309570e-09};
  for (double x0 : starts) {
    const uint64_t b = dvh::rng::double_to_bits(x0);
    for (long long d = -sweep / 2; d < sweep / 2; ++d) {
      const double x = dvh::rng::bits_to_double(b + (uint64_t)(d * 1024));
      if (x > -1.0 && x < 1.0) check(x);
    }
  }
  return bad;
}
}

// dvh_series.hip -- the synthetic scenario sweep's inputs generated in HBM (BASELINE.json configs 4 / 5, SURVEY.md
// 8d; dervet_hip/lp/scenarios.py sweep_parameters / _config4_series / windows_by_period + gpu_builder
// battery_group_spec).  Before this, a 10,000-scenario sweep spent ~4 s on the host drawing 87.6 M normals, filtering
// them and cutting the windows' series, against ~0.55 s of solve.
//
// series_draws_kernel: one thread per scenario runs the scenario's PCG64 stream exactly as numpy does (dvh_rng.h):
//   load scale's normal, 8,760 normals through the AR(1) filter as scipy.signal.lfilter([1], [1, -phi]) evaluates it
//   (y = z + x; z = x * 0 - y * a1, the innovations after the first scaled by sqrt(1 - phi^2)), then the uniform
//   draws' next_double words.  The host finishes the scalars (exp for the lognormal with the host libm, low + range
//   * u for the uniforms: 10,000 x 7 numbers).
// series_windows_kernel: one workgroup per window forms the device builder's inputs for a window of a scenario --
//   base = load - PV + hp, retail = price x price scale -- and the window's objective constant as numpy sums it
//   (in order, or pairwise for a lone window), so every array equals the host spec's bit for bit
//   (tests/test_gpu_series.py).
#include <math.h>

#include "../../include/dervet_hip.h"
// Bit-identity with numpy: every operation rounded on its own, no FMA contraction in this file.
#pragma clang fp contract(off)
#include "dvh_internal.h"
#include "dvh_rng.h"

namespace dvh {
namespace {

constexpr int kDrawB = 64;
constexpr int kWinB = 256;

struct DeviceExp {
  __device__ double operator()(double v) const { return exp(v); }
};

__global__ __launch_bounds__(kDrawB) void series_draws_kernel(const uint64_t* seeds, int count, int steps, int n_unif,
                                                             double a1, double innov, double* z0, double* ar,
                                                             double* unif, int32_t* ambiguous,
                                                             int32_t* amb_rows) {
  const int i = blockIdx.x * kDrawB + threadIdx.x;
  if (i >= count) return;
  rng::Pcg64 g = rng::seed_pcg64(seeds[i]);
  int amb = 0;
  const DeviceExp ex;
  z0[i] = rng::normal(g, ex, amb);
  double* out = ar + (int64_t)i * steps;
  double z = 0.0;  // lfilter's delay state (zi = 0)
  for (int t = 0; t < steps; ++t) {
    const double e = rng::normal(g, ex, amb);
    const double x = t == 0 ? e : e * innov;
    const double y = z + x;
    z = x * 0.0 - y * a1;
    out[t] = y;
  }
  for (int k = 0; k < n_unif; ++k) unif[(int64_t)i * n_unif + k] = rng::next_double(g);
  if (amb_rows) amb_rows[i] = amb ? 1 : 0;
  if (amb) atomicAdd(ambiguous, 1);
}

// numpy's pairwise sum of n <= 8192 values v(0 .. n-1) (DOUBLE_pairwise_sum): blocks of <= 128 summed with 8
// accumulators, longer ranges split at n / 2 rounded down to a multiple of 8; evaluated with an explicit stack.
template <class V>
__device__ double pairwise_sum(const V& v, int off0, int n0) {
  struct Frame {
    int off, n, stage;
    double left;
  };
  Frame st[16];
  int sp = 0;
  st[sp++] = Frame{off0, n0, 0, 0.0};
  double ret = 0.0;
  bool have = false;  // `ret` holds a finished child's value
  while (sp > 0) {
    Frame& f = st[sp - 1];
    if (f.n <= 128) {
      double res;
      if (f.n < 8) {
        res = 0.0;
        for (int i = 0; i < f.n; ++i) res = res + v(f.off + i);
      } else {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = v(f.off + j);
        int i = 8;
        for (; i < f.n - (f.n % 8); i += 8)
          for (int j = 0; j < 8; ++j) r[j] = r[j] + v(f.off + i + j);
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < f.n; ++i) res = res + v(f.off + i);
      }
      --sp;
      ret = res;
      have = true;
      continue;
    }
    int n2 = f.n / 2;
    n2 -= n2 % 8;
    if (f.stage == 0) {
      f.stage = 1;
      st[sp++] = Frame{f.off, n2, 0, 0.0};
      have = false;
    } else if (f.stage == 1) {
      f.left = ret;
      f.stage = 2;
      st[sp++] = Frame{f.off + n2, f.n - n2, 0, 0.0};
      have = false;
    } else {
      const double val = f.left + ret;
      --sp;
      ret = val;
      have = true;
    }
  }
  (void)have;
  return ret;
}

struct WindowProduct {  // (retail * dt) * base of a window, as numpy's (retail * dt * base) array
  const double* r;
  const double* b;
  double dt;
  __device__ double operator()(int t) const { return (r[t] * dt) * b[t]; }
};

__global__ __launch_bounds__(kWinB) void series_windows_kernel(const dvh_window_series w, int32_t* bad) {
  const int k = blockIdx.x;
  const int s = w.rows[k];
  if (s < 0 || s >= w.count) {
    if (threadIdx.x == 0) atomicAdd(bad, 1);
    return;
  }
  const double ls = w.load_scale[s], ps = w.price_scale[s], pv = w.pv_rated[s], hp = w.hp[s];
  const double* a = w.ar + (int64_t)s * w.hours;
  double* bo = w.base + (int64_t)k * w.T;
  double* ro = w.retail + (int64_t)k * w.T;
  for (int t = threadIdx.x; t < w.T; t += kWinB) {
    const int tau = w.t0 + t, hr = tau / w.rep;
    const double load = (w.site_load[hr] * ls) * (1.0 + 0.05 * a[hr]);
    const double gen = pv * w.pv_profile[hr];
    bo[t] = (load - gen) + hp;
    ro[t] = w.price[tau] * ps;
  }
  __syncthreads();  // the window's base / retail rows are visible to the whole workgroup
  if (threadIdx.x == 0) {
    // numpy's (retail * dt * base).sum(axis=1): the host series are column selections of [S, steps] arrays, so the
    // [G, T] product is Fortran-ordered and numpy reduces it with the window index innermost -- an ordered running
    // sum over t.  A lone window (G = 1) is contiguous along t, and numpy sums its row pairwise in 8,192-element
    // buffers.
    const WindowProduct v{ro, bo, w.dt};
    double acc = 0.0;  // the reduction's identity
    if (w.G == 1) {
      for (int off = 0; off < w.T; off += 8192) acc = acc + pairwise_sum(v, off, min(8192, w.T - off));
    } else {
      for (int t = 0; t < w.T; ++t) acc = acc + v(t);
    }
    // battery_group_spec's running objective constant: zeros (+ zeros per DCM group), + the retail term's sum,
    // + fixed O&M x discharge rating, + zeros (the variable O&M term's constant)
    double c0 = 0.0;
    if (w.J > 0) c0 = c0 + 0.0;
    c0 = c0 + acc;
    c0 = c0 + w.c0_add[s];
    c0 = c0 + 0.0;
    w.c0[k] = c0;
  }
}

}  // namespace

hipError_t launch_series_draws(const uint64_t* seeds, int count, int steps, int n_unif, double a1, double innov,
                               double* z0, double* ar, double* unif, int32_t* ambiguous, int32_t* amb_rows,
                               hipStream_t s) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(series_draws_kernel, dim3((count + kDrawB - 1) / kDrawB), dim3(kDrawB), 0, s, seeds, count,
                     steps, n_unif, a1, innov, z0, ar, unif, ambiguous, amb_rows);
  return hipGetLastError();
}

hipError_t launch_series_windows(const dvh_window_series& w, int32_t* bad, hipStream_t s) {
  if (w.G <= 0) return hipSuccess;
  hipLaunchKernelGGL(series_windows_kernel, dim3(w.G), dim3(kWinB), 0, s, w, bad);
  return hipGetLastError();
}

}  // namespace dvh

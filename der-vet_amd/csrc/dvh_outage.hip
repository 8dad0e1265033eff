// dvh_outage.hip -- post-facto reliability sweep on gfx950: one outage simulated from every start step.
//
// Replaces the serial Python recursion of DER-VET's load-coverage-probability curve
// (dervet/MicrogridValueStreams/Reliability.py:876-967 load_coverage_probability, :447-487 data_process,
// :489-570 simulate_outage; restated for tests in oracle/outage.py).  Every (case, start step) is one
// thread: it walks the outage step by step (charge the ESS from excess generation, else discharge to cover the
// critical load) until a step fails, the data ends or the maximum outage length is reached, and records the
// covered length.  Neighbouring threads read neighbouring steps, so the per-step loads of critical load / PV /
// SOE are coalesced; a per-workgroup LDS histogram of covered lengths is flushed with one integer atomic per
// bin (integer sums: order-independent, bit-exact).
//
// Bit-exactness with the numpy reference: the arithmetic is IEEE double with no contraction (no FMA), the
// roundings are numpy.around's (x * 10^d, round half to even, / 10^d), and Python's min() is restated by
// first-smallest comparisons.
#include <hip/hip_runtime.h>
#include <math.h>

#include "dvh_internal.h"

namespace dvh {
namespace {

constexpr int kOutB = 256;

__device__ __forceinline__ double around(double x, double f) {
#pragma clang fp contract(off)
  return rint(x * f) / f;
}
// Python min(a, b, c): the first smallest argument
__device__ __forceinline__ double pymin3(double a, double b, double c) {
  double r = a;
  if (b < r) r = b;
  if (c < r) r = c;
  return r;
}

// MINSOE = false: covered length per start + histogram (load_coverage_probability :876-967).
// MINSOE = true: soe_used per start = max - min of the SOE profile including the start (min_soe_iterative
// :685-756, the reliability minimum-SOE requirement), written to soe_used[len_off + t].
template <bool MINSOE>
__global__ __launch_bounds__(kOutB) void outage_kernel(const OutageCase* cases, int32_t* lengths, int32_t* hist,
                                                      double* soe_used) {
#pragma clang fp contract(off)
  extern __shared__ int32_t lh[];  // [outage_len + 1] histogram of this workgroup
  const OutageCase c = cases[blockIdx.y];
  const int nb = c.outage_len + 1;
  if (!MINSOE) {
    for (int i = threadIdx.x; i < nb; i += kOutB) lh[i] = 0;
    __syncthreads();
  }
  const int t = blockIdx.x * kOutB + threadIdx.x;
  if (t < c.n_steps) {
    const int stop = min(t + c.max_steps, c.n_steps);  // data_process slices max_steps entries (:462-465)
    double soe = (!MINSOE && c.init_soe) ? c.init_soe[t] : c.soe0;
    double smax = soe, smin = soe;
    int k = 0;
    for (; k < c.outage_len; ++k) {
      const int i = t + k;
      if (i >= stop) break;  // no data left (:524)
      double cl = c.critical_load[i];
      if (c.load_shed) cl = cl * (c.load_shed[k] / 100.0);
      const double g = c.dg_gen;
      const double pm = c.pv_max ? c.pv_max[i] : 0.0, pv = c.pv_vari ? c.pv_vari[i] : 0.0;
      const double dl = around(cl - g - pm, 1e5);
      const double rc = around(cl - g - pv, 1e5);
      const double ec = rc * c.gamma;
      if (0.0 >= rc) {  // excess generation: charge if there is room (:529-541)
        if (c.soe_max >= soe) {
          const double charge_possible = (c.soe_max - soe) / (c.rte * c.dt);
          const double charge = pymin3(charge_possible, -dl, c.charge_max);
          soe = soe + (charge * c.rte * c.dt);
        }
      } else {  // discharge to cover the load (:544-564)
        if (!(0.0 >= around(ec * c.dt - soe, 1e2))) break;
        const double discharge_possible = (soe - c.soe_min) / c.dt;
        const double discharge = pymin3(discharge_possible, dl, c.discharge_max);
        if (0.0 < around(dl - discharge, 1e2)) break;
        soe = soe - (discharge * c.dt);
      }
      if (MINSOE) {
        smax = soe > smax ? soe : smax;
        smin = soe < smin ? soe : smin;
      }
    }
    if (MINSOE) {
      soe_used[c.len_off + t] = smax - smin;
    } else {
      if (lengths) lengths[c.len_off + t] = k;
      atomicAdd(&lh[k], 1);
    }
  }
  if (!MINSOE) {
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += kOutB)
      if (lh[i]) atomicAdd(&hist[c.hist_off + i], lh[i]);
  }
}

}  // namespace

hipError_t launch_outage(const OutageCase* d_cases, int ncase, int max_steps_n, int max_bins, int32_t* d_lengths,
                         int32_t* d_hist, hipStream_t s) {
  if (ncase <= 0 || max_steps_n <= 0) return hipSuccess;
  const size_t lds = sizeof(int32_t) * (size_t)max_bins;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  dim3 grid((max_steps_n + kOutB - 1) / kOutB, ncase);
  hipLaunchKernelGGL(outage_kernel<false>, grid, dim3(kOutB), lds, s, d_cases, d_lengths, d_hist, nullptr);
  return hipGetLastError();
}

hipError_t launch_outage_min_soe(const OutageCase* d_cases, int ncase, int max_steps_n, double* d_soe_used,
                                 hipStream_t s) {
  if (ncase <= 0 || max_steps_n <= 0) return hipSuccess;
  dim3 grid((max_steps_n + kOutB - 1) / kOutB, ncase);
  hipLaunchKernelGGL(outage_kernel<true>, grid, dim3(kOutB), 0, s, d_cases, nullptr, nullptr, d_soe_used);
  return hipGetLastError();
}

}  // namespace dvh

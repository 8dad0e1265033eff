// dvh_sweep.hip -- warm starts of a seeded scenario sweep (dervet_hip/sweep.py; DER-VET's sensitivity cases,
// dervet/DERVET.py:75, solve the same windows for thousands of perturbed scenarios), in one launch.
//
// Every listed window starts from its partner window's solution (a solved seed of the same window id and CSR
// pattern): x scaled per column by the ratio of the two windows' upper bounds where both are finite and the
// partner's is positive (charge / discharge power, energy rating), else copied; for the battery + DCM shape
// (x = [ch, dis, ene, tau], one demand column) the duals of the init / SOE rows scaled by the ratio of the windows'
// mean |c| over the ch columns (energy prices) and those of the DCM rows by the ratio of the demand charges (c of
// tau), else copied.  One 256-thread workgroup per window; reads the partners' x / y, writes the windows'.
#include "dvh_internal.h"

namespace dvh {
namespace {

constexpr int kSwB = 256;

__global__ __launch_bounds__(kSwB) void warm_transfer_kernel(const int64_t* desc, const double* c, const double* u,
                                                             double* x, double* y, const int32_t* pairs,
                                                             int32_t* bad) {
  __shared__ double red[2 * (kSwB / kWave)];
  const int w = pairs[3 * blockIdx.x], p = pairs[3 * blockIdx.x + 1], T = pairs[3 * blockIdx.x + 2];
  const int64_t* dw = desc + 8 * (int64_t)w;
  const int64_t* dp = desc + 8 * (int64_t)p;
  const int64_t n = dw[0], m = dw[1];
  if (n != dp[0] || m != dp[1] || (T > 0 && (3 * (int64_t)T + 1 != n || T + 1 > m))) {  // not the same shape
    if (threadIdx.x == 0) atomicAdd(bad, 1);
    return;
  }
  const int64_t onw = dw[6], omw = dw[7], onp = dp[6], omp = dp[7];
  const int tid = threadIdx.x;
  for (int64_t j = tid; j < n; j += kSwB) {
    const double ur = u[onw + j], us = u[onp + j];
    const bool ok = isfinite(ur) && isfinite(us) && us > 0.0;
    x[onw + j] = x[onp + j] * (ok ? ur / us : 1.0);
  }
  if (T <= 0) {
    for (int64_t i = tid; i < m; i += kSwB) y[omw + i] = y[omp + i];
    return;
  }
  // mean |c| over the ch columns of both windows (fixed-order block sums)
  double a = 0.0, b = 0.0;
  for (int j = tid; j < T; j += kSwB) {
    a += fabs(c[onw + j]);
    b += fabs(c[onp + j]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, kWave);
    b += __shfl_xor(b, o, kWave);
  }
  const int lane = tid & 63, wid = tid >> 6;
  if (lane == 0) {
    red[2 * wid] = a;
    red[2 * wid + 1] = b;
  }
  __syncthreads();
  double sa = 0.0, sb = 0.0;
  for (int v = 0; v < kSwB / kWave; ++v) {
    sa += red[2 * v];
    sb += red[2 * v + 1];
  }
  const double cp = (sa / T) / fmax(sb / T, 1e-12);
  const double cd = c[onw + 3 * (int64_t)T] / fmax(c[onp + 3 * (int64_t)T], 1e-12);
  for (int64_t i = tid; i < m; i += kSwB) y[omw + i] = y[omp + i] * (i <= T ? cp : cd);
}

}  // namespace

hipError_t launch_warm_transfer(const int64_t* desc, const double* c, const double* u, double* x, double* y,
                                const int32_t* pairs, int count, int32_t* bad, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(warm_transfer_kernel, dim3(count), dim3(kSwB), 0, s, desc, c, u, x, y, pairs, bad);
  return hipGetLastError();
}

}  // namespace dvh

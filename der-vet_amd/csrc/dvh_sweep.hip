// dvh_sweep.hip -- warm starts of a seeded scenario sweep (dervet_hip/sweep.py; DER-VET's sensitivity cases,
// dervet/DERVET.py:75, solve the same windows for thousands of perturbed scenarios), in one launch.
//
// Every listed window starts from its partner window's solution (a solved seed of the same window id and CSR
// pattern): x scaled per column by the ratio of the two windows' upper bounds where both are finite and the
// partner's is positive (charge / discharge power, energy rating), else copied; for the battery + DCM shape
// (x = [ch, dis, ene, tau], one demand column) the duals of the init / SOE rows scaled by the ratio of the windows'
// mean |c| over the ch columns (energy prices) and those of the DCM rows by the ratio of the demand charges (c of
// tau), else copied.  One 256-thread workgroup per window; reads the partners' x / y, writes the windows'.  A window
// may also start from a weighted blend of several partners' transferred solutions (dvh_warm_transfer_blend: the
// seeded sweep's nearest seeds, inverse-distance weights).
#include "dvh_internal.h"

namespace dvh {
namespace {

constexpr int kSwB = 256;

// rows[(Q + 2) b] = {window, partner_1 .. partner_Q, T}; wts[Q b] the partners' weights (sum 1).  x = sum_i w_i x_i',
// y = sum_i w_i y_i' with x_i', y_i' partner i's solution transferred as above (partners summed in list order).  Q = 1
// with weight 1 is the single-partner transfer bit for bit (1 * v + 0 == v).
__global__ __launch_bounds__(kSwB) void warm_transfer_kernel(const int64_t* desc, const double* c, const double* u,
                                                             double* x, double* y, const int32_t* rows,
                                                             const double* wts, int Q, int32_t* bad) {
  __shared__ double red[(kMaxBlend + 1) * (kSwB / kWave)];
  __shared__ double cps[kMaxBlend], cds[kMaxBlend];
  const int32_t* row = rows + (int64_t)(Q + 2) * blockIdx.x;
  const int w = row[0], T = row[Q + 1];
  const int64_t* dw = desc + 8 * (int64_t)w;
  const int64_t n = dw[0], m = dw[1];
  bool ok_shape = !(T > 0 && (3 * (int64_t)T + 1 != n || T + 1 > m));
  for (int i = 0; i < Q; ++i) {
    const int64_t* dp = desc + 8 * (int64_t)row[1 + i];
    ok_shape &= n == dp[0] && m == dp[1];
  }
  if (!ok_shape) {  // not the same shape
    if (threadIdx.x == 0) atomicAdd(bad, 1);
    return;
  }
  const double* wq = wts + (int64_t)Q * blockIdx.x;
  const int64_t onw = dw[6], omw = dw[7];
  const int tid = threadIdx.x;
  for (int64_t j = tid; j < n; j += kSwB) {
    const double ur = u[onw + j];
    double acc = 0.0;
    for (int i = 0; i < Q; ++i) {
      const int64_t onp = desc[8 * (int64_t)row[1 + i] + 6];
      const double us = u[onp + j];
      const bool ok = isfinite(ur) && isfinite(us) && us > 0.0;
      acc += wq[i] * (x[onp + j] * (ok ? ur / us : 1.0));
    }
    x[onw + j] = acc;
  }
  if (T <= 0) {
    for (int64_t i = tid; i < m; i += kSwB) {
      double acc = 0.0;
      for (int q = 0; q < Q; ++q) acc += wq[q] * y[desc[8 * (int64_t)row[1 + q] + 7] + i];
      y[omw + i] = acc;
    }
    return;
  }
  // mean |c| over the ch columns of the window and of every partner (fixed-order block sums)
  const int lane = tid & 63, wid = tid >> 6;
  double a = 0.0;
  double bq[kMaxBlend];
  for (int q = 0; q < kMaxBlend; ++q) bq[q] = 0.0;
  for (int j = tid; j < T; j += kSwB) {
    a += fabs(c[onw + j]);
    for (int q = 0; q < Q; ++q) bq[q] += fabs(c[desc[8 * (int64_t)row[1 + q] + 6] + j]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, kWave);
    for (int q = 0; q < Q; ++q) bq[q] += __shfl_xor(bq[q], o, kWave);
  }
  if (lane == 0) {
    red[(kMaxBlend + 1) * wid] = a;
    for (int q = 0; q < Q; ++q) red[(kMaxBlend + 1) * wid + 1 + q] = bq[q];
  }
  __syncthreads();
  if (tid < Q) {
    double sa = 0.0, sb = 0.0;
    for (int v = 0; v < kSwB / kWave; ++v) {
      sa += red[(kMaxBlend + 1) * v];
      sb += red[(kMaxBlend + 1) * v + 1 + tid];
    }
    const int64_t onp = desc[8 * (int64_t)row[1 + tid] + 6];
    cps[tid] = (sa / T) / fmax(sb / T, 1e-12);
    cds[tid] = c[onw + 3 * (int64_t)T] / fmax(c[onp + 3 * (int64_t)T], 1e-12);
  }
  __syncthreads();
  for (int64_t i = tid; i < m; i += kSwB) {
    double acc = 0.0;
    for (int q = 0; q < Q; ++q)
      acc += wq[q] * (y[desc[8 * (int64_t)row[1 + q] + 7] + i] * (i <= T ? cps[q] : cds[q]));
    y[omw + i] = acc;
  }
}

}  // namespace

hipError_t launch_warm_transfer(const int64_t* desc, const double* c, const double* u, double* x, double* y,
                                const int32_t* rows, const double* wts, int q, int count, int32_t* bad, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  if (q < 1 || q > kMaxBlend) return hipErrorInvalidValue;
  hipLaunchKernelGGL(warm_transfer_kernel, dim3(count), dim3(kSwB), 0, s, desc, c, u, x, y, rows, wts, q, bad);
  return hipGetLastError();
}

}  // namespace dvh

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
  // the partners' offsets and weights, loaded once (uniform; slots q >= Q unused)
  int64_t onp[kMaxBlend], omp[kMaxBlend];
  double wqv[kMaxBlend];
#pragma unroll
  for (int q = 0; q < kMaxBlend; ++q) {
    const int64_t* dp = desc + 8 * (int64_t)row[1 + (q < Q ? q : 0)];
    onp[q] = dp[6];
    omp[q] = dp[7];
    wqv[q] = q < Q ? wq[q] : 0.0;
  }
  // [r5] every load of a chunk of kU elements per thread is issued before its arithmetic and stores (the window's
  // x / y never overlap a partner's: a partner is a solved seed, never a listed window), so a thread has 2 kU Q loads
  // in flight instead of one element's; the arithmetic per element is unchanged (bit-identical results)
  constexpr int kU = 2;
  for (int64_t j0 = tid; j0 < n; j0 += kU * kSwB) {
    double ur[kU], uv[kMaxBlend][kU], xv[kMaxBlend][kU];
#pragma unroll
    for (int e = 0; e < kU; ++e) {
      const int64_t j = j0 + e * kSwB;
      ur[e] = j < n ? u[onw + j] : 0.0;
#pragma unroll
      for (int q = 0; q < kMaxBlend; ++q) {
        uv[q][e] = (q < Q && j < n) ? u[onp[q] + j] : 1.0;
        xv[q][e] = (q < Q && j < n) ? x[onp[q] + j] : 0.0;
      }
    }
#pragma unroll
    for (int e = 0; e < kU; ++e) {
      const int64_t j = j0 + e * kSwB;
      if (j >= n) break;
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < kMaxBlend; ++q) {
        if (q >= Q) break;
        const double us = uv[q][e];
        const bool ok = isfinite(ur[e]) && isfinite(us) && us > 0.0;
        acc += wqv[q] * (xv[q][e] * (ok ? ur[e] / us : 1.0));
      }
      x[onw + j] = acc;
    }
  }
  if (T <= 0) {
    for (int64_t i = tid; i < m; i += kSwB) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < kMaxBlend; ++q) {
        if (q >= Q) break;
        acc += wqv[q] * y[omp[q] + i];
      }
      y[omw + i] = acc;
    }
    return;
  }
  // mean |c| over the ch columns of the window and of every partner (fixed-order block sums)
  const int lane = tid & 63, wid = tid >> 6;
  double a = 0.0;
  double bq[kMaxBlend];
#pragma unroll
  for (int q = 0; q < kMaxBlend; ++q) bq[q] = 0.0;
  for (int j = tid; j < T; j += kSwB) {
    a += fabs(c[onw + j]);
#pragma unroll
    for (int q = 0; q < kMaxBlend; ++q)
      if (q < Q) bq[q] += fabs(c[onp[q] + j]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, kWave);
#pragma unroll
    for (int q = 0; q < kMaxBlend; ++q)
      if (q < Q) bq[q] += __shfl_xor(bq[q], o, kWave);
  }
  if (lane == 0) {
    red[(kMaxBlend + 1) * wid] = a;
#pragma unroll
    for (int q = 0; q < kMaxBlend; ++q)
      if (q < Q) red[(kMaxBlend + 1) * wid + 1 + q] = bq[q];
  }
  __syncthreads();
  if (tid < Q) {
    double sa = 0.0, sb = 0.0;
    for (int v = 0; v < kSwB / kWave; ++v) {
      sa += red[(kMaxBlend + 1) * v];
      sb += red[(kMaxBlend + 1) * v + 1 + tid];
    }
    const int64_t onq = desc[8 * (int64_t)row[1 + tid] + 6];
    cps[tid] = (sa / T) / fmax(sb / T, 1e-12);
    cds[tid] = c[onw + 3 * (int64_t)T] / fmax(c[onq + 3 * (int64_t)T], 1e-12);
  }
  __syncthreads();
  double cp[kMaxBlend], cd[kMaxBlend];
#pragma unroll
  for (int q = 0; q < kMaxBlend; ++q) {
    cp[q] = q < Q ? cps[q] : 0.0;
    cd[q] = q < Q ? cds[q] : 0.0;
  }
  for (int64_t i0 = tid; i0 < m; i0 += kU * kSwB) {
    double yv[kMaxBlend][kU];
#pragma unroll
    for (int e = 0; e < kU; ++e) {
      const int64_t i = i0 + e * kSwB;
#pragma unroll
      for (int q = 0; q < kMaxBlend; ++q) yv[q][e] = (q < Q && i < m) ? y[omp[q] + i] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < kU; ++e) {
      const int64_t i = i0 + e * kSwB;
      if (i >= m) break;
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < kMaxBlend; ++q) {
        if (q >= Q) break;
        acc += wqv[q] * (yv[q][e] * (i <= T ? cp[q] : cd[q]));
      }
      y[omw + i] = acc;
    }
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

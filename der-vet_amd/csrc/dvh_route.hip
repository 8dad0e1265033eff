// dvh_route.hip -- the kernel cascade's window lists formed on the device (dvh_api.cpp solve_packed).
//
// Each on-chip tier hands the windows it cannot take to the next one by their status: the battery-banded kernel
// writes kNeedsEll (-2), the ELL kernel kNeedsGeneric (-1).  The next tier's list used to be built on the host from
// a read-back of every window's status (one host sync and an O(windows) host loop per tier).  route_kernel builds it
// in HBM instead, in window order (the tiers' results do not depend on it, the order only keeps runs reproducible to
// read): one 1024-thread workgroup, each thread a contiguous range of the input, counts -> block exclusive scan ->
// ordered writes.  It also reduces the listed windows' sizes (n, m, nnz) and ELL widths (the setup kernel's
// per-window statistics), from which the host picks the next tier's instantiation -- sized for the windows that
// reach it, not for the whole chunk, and split by size class (a mixed batch's market days take the small ELL
// kernels; windows no ELL instantiation holds go to the generic kernel without dragging them along) -- so one small
// read-back replaces the status and statistics copies.
#include "dvh_internal.h"

namespace dvh {
namespace {

constexpr int kRouteB = 1024;

// out_info: [0] listed windows, [1] max wx, [2] max wy (ELL widths over the listed windows the setup kernel scaled),
// [3] max n, [4] max m, [5] max nnz (over the listed windows)
// cls: 0 every size up to small_max, 1 only n <= lim_n and m <= lim_m, 2 only the others
__global__ __launch_bounds__(kRouteB) void route_kernel(const int64_t* desc, const int32_t* istats, const double* scal,
                                                       int first, int count, const int32_t* in_list, int want,
                                                       int small_max, int cls, int lim_n, int lim_m,
                                                       int32_t* out_list, int32_t* out_info) {
  constexpr int NV = 5;
  __shared__ int32_t part[kRouteB];
  __shared__ int32_t wmax[NV][kRouteB / kWave];
  const int tid = threadIdx.x;
  const int per = (count + kRouteB - 1) / kRouteB;
  const int a = min(count, tid * per), e = min(count, a + per);
  auto window = [&](int i) { return in_list ? in_list[i] : first + i; };
  auto match = [&](int k) {
    const int64_t* d = desc + 8 * (int64_t)k;
    if (d[0] > small_max || d[1] > small_max || istats[2 * (int64_t)k] != want) return false;
    const bool in_lim = d[0] <= lim_n && d[1] <= lim_m;
    return cls == 0 || (cls == 1) == in_lim;
  };
  int cnt = 0, v[NV] = {0, 0, 0, 0, 0};  // wx, wy, n, m, nnz
  for (int i = a; i < e; ++i) {
    const int k = window(i);
    if (!match(k)) continue;
    ++cnt;
    const int64_t* d = desc + 8 * (int64_t)k;
    v[2] = max(v[2], (int)d[0]);
    v[3] = max(v[3], (int)d[1]);
    v[4] = max(v[4], (int)d[3]);
    const double* sc = scal + (int64_t)(k - first) * kScal;
    if (sc[6] == 0.0) {
      v[0] = max(v[0], (int)sc[9]);
      v[1] = max(v[1], (int)sc[8]);
    }
  }
  // block exclusive scan of the counts (Hillis-Steele over LDS; 10 steps)
  part[tid] = cnt;
  __syncthreads();
  for (int off = 1; off < kRouteB; off <<= 1) {
    const int add = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += add;
    __syncthreads();
  }
  int pos = part[tid] - cnt;
  for (int i = a; i < e; ++i) {
    const int k = window(i);
    if (match(k)) out_list[pos++] = k;
  }
  // maxima: wave reductions, then thread 0
  const int lane = tid & (kWave - 1), wv = tid / kWave;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    for (int o = kWave / 2; o > 0; o >>= 1) v[u] = max(v[u], __shfl_xor(v[u], o));
    if (lane == 0) wmax[u][wv] = v[u];
  }
  __syncthreads();
  if (tid == 0) {
    out_info[0] = part[kRouteB - 1];
    for (int u = 0; u < NV; ++u) {
      int mx = 0;
      for (int q = 0; q < kRouteB / kWave; ++q) mx = max(mx, wmax[u][q]);
      out_info[1 + u] = mx;
    }
  }
}

}  // namespace

hipError_t launch_route(const int64_t* desc, const int32_t* istats, const double* scal, int first, int count,
                        const int32_t* in_list, int want, int small_max, int cls, int lim_n, int lim_m,
                        int32_t* out_list, int32_t* out_info, hipStream_t s) {
  hipLaunchKernelGGL(route_kernel, dim3(1), dim3(kRouteB), 0, s, desc, istats, scal, first, count, in_list, want,
                     small_max, cls, lim_n, lim_m, out_list, out_info);
  return hipGetLastError();
}

}  // namespace dvh

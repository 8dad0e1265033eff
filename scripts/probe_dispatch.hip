// probe_dispatch.hip -- does the workgroup dispatcher lose throughput when one launch's workgroups have very different
// durations?  (dev probe for the band kernel's launch order, profiles/r04p_ab_launch_order.log: the same windows ran
// 7-8 % faster launched sorted by duration, either direction.)
//
// Synthetic kernel: 256 threads, 74 KB of dynamic LDS (two workgroups per CU, as the band kernel's three-step form),
// each workgroup spins for its own duration (s_memrealtime ticks, 100 MHz) drawn from the bench's warm-phase
// iteration counts' shape (log-normal, mean ~1.9 ms).  Variants:
//   packed   -- one workgroup per item, items in random order
//   sorted   -- the same items sorted by duration (descending)
//   queue    -- persistent: CUs x 2 workgroups taking items from an atomic counter
//   xcdN     -- N CU-masked streams (hipExtStreamCreateWithCUMask), items split round-robin over them
// Also prints which XCD (HW_REG_XCC_ID) each stream's workgroups ran on.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/_variants/probe_dispatch scripts/probe_dispatch.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int kB = 256;
constexpr size_t kLds = 74 * 1024;

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}
__device__ __forceinline__ uint64_t now() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

__device__ void spin(uint64_t ticks, double* sink) {
  extern __shared__ double lds[];
  const uint64_t t0 = now();
  double a = threadIdx.x;
  for (int guard = 0; guard < (1 << 22) && now() - t0 < ticks; ++guard) a = a * 0.999999 + 1e-9;
  lds[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) sink[0] += lds[1] * 0.0;
}

__global__ __launch_bounds__(kB) void one_each(const uint32_t* ticks, const int32_t* list, int count, double* sink,
                                               int32_t* xcc) {
  const int i = list ? list[blockIdx.x] : blockIdx.x;
  if (threadIdx.x == 0 && xcc) xcc[blockIdx.x] = xcc_id();
  spin(ticks[i], sink);
}

__global__ __launch_bounds__(kB) void persistent(const uint32_t* ticks, int count, int32_t* queue, double* sink) {
  __shared__ int next;
  for (;;) {
    // wave 0 takes the next item: a wave-uniform branch, the whole wave in the atomic (lane 0 adds 1, the others 0).
    // A lane-0-only atomic (if (threadIdx.x == 0)) inside the loop was structurized into an inner loop whose barriers
    // the waves no longer reached in step: the workgroups hung.
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) < 64)
      next = __builtin_amdgcn_readfirstlane(atomicAdd(queue, (threadIdx.x & 63) == 0 ? 1 : 0));
    __syncthreads();
    const int i = __builtin_amdgcn_readfirstlane(next);
    __syncthreads();
    if (i >= count) return;
    spin(ticks[i], sink);
  }
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int count = argc > 1 ? atoi(argv[1]) : 30000;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipFuncSetAttribute((const void*)one_each, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds));
  CHECK(hipFuncSetAttribute((const void*)persistent, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds));
  int nb = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)one_each, kB, kLds));
  printf("CUs %d, resident workgroups per CU %d, items %d\n", cus, nb, count);
  // durations: log-normal with the warm phase's spread (median ~1,650 iterations, p99 ~4,700) at ~1 us per iteration,
  // scaled down 4x so a launch takes ~100 ms
  std::mt19937_64 rng(7);
  std::lognormal_distribution<double> ln(std::log(1650.0), 0.55);
  std::vector<uint32_t> ticks(count);
  double total = 0;
  for (auto& t : ticks) {
    const double us = std::min(ln(rng), 11000.0) / 4.0;
    t = (uint32_t)(us * 100.0);  // 100 MHz ticks
    total += us;
  }
  printf("ideal makespan %.2f ms (sum / slots)\n", total / 1000.0 / (cus * nb));
  uint32_t* d_ticks;
  int32_t *d_list, *d_queue, *d_xcc;
  double* d_sink;
  CHECK(hipMalloc(&d_ticks, 4 * count));
  CHECK(hipMalloc(&d_list, 4 * count));
  CHECK(hipMalloc(&d_queue, 4));
  CHECK(hipMalloc(&d_xcc, 4 * count));
  CHECK(hipMalloc(&d_sink, 8));
  CHECK(hipMemcpy(d_ticks, ticks.data(), 4 * count, hipMemcpyHostToDevice));
  std::vector<int32_t> sorted(count);
  for (int i = 0; i < count; ++i) sorted[i] = i;
  std::sort(sorted.begin(), sorted.end(), [&](int a, int b) { return ticks[a] > ticks[b]; });
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timed = [&](const char* name, auto fn) {
    fn();  // warm-up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    fn();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-10s %8.2f ms\n", name, ms);
  };
  timed("packed", [&] { hipLaunchKernelGGL(one_each, dim3(count), dim3(kB), kLds, 0, d_ticks, nullptr, count, d_sink, nullptr); });
  CHECK(hipMemcpy(d_list, sorted.data(), 4 * count, hipMemcpyHostToDevice));
  timed("sorted", [&] { hipLaunchKernelGGL(one_each, dim3(count), dim3(kB), kLds, 0, d_ticks, d_list, count, d_sink, nullptr); });
  timed("queue", [&] {
    CHECK(hipMemsetAsync(d_queue, 0, 4, 0));
    hipLaunchKernelGGL(persistent, dim3(cus * nb), dim3(kB), kLds, 0, d_ticks, count, d_queue, d_sink);
  });
  // CU-masked streams: N masks over the CU bits, interleaved (bit i -> stream i % N) or contiguous
  for (int layout = 0; layout < 2; ++layout) {
    for (int N : {2, 4, 8}) {
      std::vector<hipStream_t> st(N);
      const int words = (cus + 31) / 32;
      for (int sidx = 0; sidx < N; ++sidx) {
        std::vector<uint32_t> mask(words, 0);
        for (int c = 0; c < cus; ++c) {
          const int owner = layout == 0 ? c % N : c / ((cus + N - 1) / N);
          if (owner == sidx) mask[c / 32] |= 1u << (c % 32);
        }
        CHECK(hipExtStreamCreateWithCUMask(&st[sidx], words, mask.data()));
      }
      // items split round-robin over the streams (each stream: its own sub-list, packed order)
      std::vector<std::vector<int32_t>> sub(N);
      for (int i = 0; i < count; ++i) sub[i % N].push_back(i);
      std::vector<int32_t*> d_sub(N);
      for (int sidx = 0; sidx < N; ++sidx) {
        CHECK(hipMalloc(&d_sub[sidx], 4 * sub[sidx].size()));
        CHECK(hipMemcpy(d_sub[sidx], sub[sidx].data(), 4 * sub[sidx].size(), hipMemcpyHostToDevice));
      }
      char name[32];
      snprintf(name, sizeof name, "%s%d", layout == 0 ? "ilv" : "blk", N);
      timed(name, [&] {
        for (int sidx = 0; sidx < N; ++sidx)
          hipLaunchKernelGGL(one_each, dim3(sub[sidx].size()), dim3(kB), kLds, st[sidx], d_ticks, d_sub[sidx],
                             (int)sub[sidx].size(), d_sink, nullptr);
        for (int sidx = 0; sidx < N; ++sidx) CHECK(hipStreamSynchronize(st[sidx]));
      });
      // XCD placement of each stream's workgroups (a short launch)
      for (int sidx = 0; sidx < N; ++sidx) {
        const int nbk = 512;
        hipLaunchKernelGGL(one_each, dim3(nbk), dim3(kB), kLds, st[sidx], d_ticks, nullptr, nbk, d_sink, d_xcc);
        CHECK(hipStreamSynchronize(st[sidx]));
        std::vector<int32_t> x(nbk);
        CHECK(hipMemcpy(x.data(), d_xcc, 4 * nbk, hipMemcpyDeviceToHost));
        int hist[16] = {0};
        for (int v : x) hist[v & 15]++;
        printf("   stream %d XCDs:", sidx);
        for (int h = 0; h < 8; ++h) printf(" %d", hist[h]);
        printf("\n");
      }
      for (int sidx = 0; sidx < N; ++sidx) {
        CHECK(hipFree(d_sub[sidx]));
        CHECK(hipStreamDestroy(st[sidx]));
      }
    }
  }
  CHECK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}

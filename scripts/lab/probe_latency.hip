// Dev microbenchmark (gfx950): dependent-chain latencies of the instructions on the band kernel's critical path.
// One workgroup of 256 threads (4 waves, one per SIMD); wave 0 times each chain with s_memtime; printed per op.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/lab/probe_latency scripts/lab/probe_latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP16(x) x x x x x x x x x x x x x x x x
__global__ void lat(double* out, unsigned long long* t, double a0) {
  __shared__ double sh[512];
  const int tid = threadIdx.x;
  double a = a0 + tid, b = 1.0000001, c = 1e-9, d = a0 * 2.0, e = a0 * 3.0, f = a0 * 4.0;
  sh[tid] = a;
  __syncthreads();
  unsigned long long t0, t1;
  int k = 0;
#define STAMP(body, n)                                                   \
  __syncthreads();                                                       \
  t0 = __builtin_amdgcn_s_memtime();                                     \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                     \
  body;                                                                  \
  asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");            \
  t1 = __builtin_amdgcn_s_memtime();                                     \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                     \
  if (tid == 0) t[k] = (t1 - t0) / (n);                                  \
  ++k;
  // 0: dependent v_fma_f64 chain (64)
  STAMP(for (int i = 0; i < 4; ++i) asm volatile(REP16("v_fma_f64 %0, %0, %1, %2\n") : "+v"(a) : "v"(b), "v"(c)), 64);
  // 1: four independent chains interleaved (64 each)
  STAMP(for (int i = 0; i < 4; ++i) asm volatile(REP16("v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5\n") : "+v"(a), "+v"(d), "+v"(e), "+v"(f) : "v"(b), "v"(c)), 256);
  // 2: dependent v_max_f64 chain alternating with v_min_f64 (64)
  STAMP(for (int i = 0; i < 4; ++i) asm volatile(REP16("v_max_f64 %0, %0, %1\n v_min_f64 %0, %0, %2\n") : "+v"(a) : "v"(c), "v"(d)), 128);
  // 3: dependent v_add_f64 chain (64)
  STAMP(for (int i = 0; i < 4; ++i) asm volatile(REP16("v_add_f64 %0, %0, %1\n") : "+v"(a) : "v"(c)), 64);
  // 4: dpp row_ror:1 of both halves + add, dependent (16)
  STAMP(for (int i = 0; i < 16; ++i) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(a), 0x121, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(a), 0x121, 0xf, 0xf, false);
    a += __hiloint2double(hi, lo);
    asm volatile("" : "+v"(a));
  }, 16);
  // 5: LDS store + read back by the neighbour lane, dependent (16)
  {
    const unsigned wa = (unsigned)(size_t)(&sh[tid]), ra = (unsigned)(size_t)(&sh[(tid + 1) & 255]);
    STAMP(for (int i = 0; i < 16; ++i) asm volatile("ds_write_b64 %1, %0\n s_waitcnt lgkmcnt(0)\n ds_read_b64 %0, %2\n s_waitcnt lgkmcnt(0)\n" : "+v"(a) : "v"(wa), "v"(ra)), 16);
  }
  // 6: LDS read only (dependent through the address? no: fixed address), issue + wait, 16
  {
    const unsigned ra = (unsigned)(size_t)(&sh[(tid + 1) & 255]);
    STAMP(for (int i = 0; i < 16; ++i) asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)\n" : "=v"(e) : "v"(ra)), 16);
  }
  // 7: barrier alone (all 4 waves arrive together), 16
  STAMP(for (int i = 0; i < 16; ++i) asm volatile("s_barrier" ::: "memory"), 16);
  // 8: readlane of a double -> v_fma with the SGPR operand, dependent (16)
  STAMP(for (int i = 0; i < 16; ++i) { double s_; asm volatile("v_readlane_b32 %0, %2, 0\n v_readlane_b32 %1, %3, 0\n" : "=s"(((unsigned*)&s_)[0]), "=s"(((unsigned*)&s_)[1]) : "v"(((unsigned*)&a)[0]), "v"(((unsigned*)&a)[1])); asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a) : "s"(s_), "v"(c)); }, 16);
  // 9: v_fma_f64 clamp chain (64)
  STAMP(for (int i = 0; i < 4; ++i) asm volatile(REP16("v_fma_f64 %0, %0, %1, %2 clamp\n") : "+v"(a) : "v"(b), "v"(c)), 64);
  // 10: v_mul_f64 chain (64)
  STAMP(for (int i = 0; i < 4; ++i) asm volatile(REP16("v_mul_f64 %0, %0, %1\n") : "+v"(a) : "v"(b)), 64);
  // 11: two independent chains interleaved (64 each)
  STAMP(for (int i = 0; i < 4; ++i) asm volatile(REP16("v_fma_f64 %0, %0, %2, %3\n v_fma_f64 %1, %1, %2, %3\n") : "+v"(a), "+v"(d) : "v"(b), "v"(c)), 128);
  out[tid] = a + d + e + f;
}

int main() {
  double* out;
  unsigned long long* t;
  hipMalloc(&out, 256 * sizeof(double));
  hipMalloc(&t, 64 * sizeof(unsigned long long));
  const char* names[] = {"fma64 dep", "fma64 4 indep", "max/min64 dep", "add64 dep", "dpp pair+add64 dep",
                         "lds write+read nbr", "lds read+wait", "barrier (4 waves)", "readlane2->fma64 dep",
                         "fma64 clamp dep", "mul64 dep", "fma64 2 indep"};
  for (int rep = 0; rep < 3; ++rep) {
    for (int blocks : {1, 512}) {
      hipLaunchKernelGGL(lat, dim3(blocks), dim3(256), 0, 0, out, t, 1.0);
      hipDeviceSynchronize();
      unsigned long long h[12];
      hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost);
      if (rep == 2) {
        printf("blocks %d:", blocks);
        for (int i = 0; i < 12; ++i) printf(" | %s %llu", names[i], h[i]);
        printf("\n");
      }
    }
  }
  return 0;
}

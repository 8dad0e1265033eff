// dvh_device.h -- device helpers shared by the PDHG kernels (dvh_kernels.hip, dvh_band.hip): DPP / permlane
// wave reductions, workgroup reductions with fixed summation order, LDS-address loads / stores, the
// primal-weight update and per-window offsets into the packed batch.
#pragma once
#include <math.h>

#include "dvh_internal.h"

namespace dvh {
namespace {

#ifndef DVH_KKT_RDX
#define DVH_KKT_RDX 1  // the objective gate's dual-residual term (kkt_done); 0: the round-3 gate (A/B builds)
#endif
constexpr int kNRed = 10 + DVH_KKT_RDX;  // values reduced by a termination (KKT) check ([10]: sum_j |r_d,j| |x_j|)
constexpr int kRdx = DVH_KKT_RDX ? 10 : 0;  // its slot (an unused 0 slot without it)
__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

constexpr int kOptimal = 0, kIterLimit = 3, kNumerical = 4;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
  return v;
}

// Wave-wide f64 sum on the VALU: DPP row rotations (16-lane rows) then the gfx950 permlane16/32 swaps.
// Every lane ends with the wave total (lanes may differ in the last bit; callers use one lane's value).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  // row rotations read every lane of the row, so the DPP "old" operand is dead: mov_dpp needs no zeroed copy
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_f64<0x128>(v);  // row_ror:8
  v += dpp_f64<0x124>(v);  // row_ror:4
  v += dpp_f64<0x122>(v);  // row_ror:2
  v += dpp_f64<0x121>(v);  // row_ror:1
  {
    const unsigned lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    v = __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
  }
  {
    const unsigned lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    v = __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
  }
  return v;
}

// Sum over each 16-lane row (every lane of the row gets its row's total; fixed order).
__device__ __forceinline__ double row_sum16(double v) {
  v += dpp_f64<0x128>(v);  // row_ror:8
  v += dpp_f64<0x124>(v);  // row_ror:4
  v += dpp_f64<0x122>(v);  // row_ror:2
  v += dpp_f64<0x121>(v);  // row_ror:1
  return v;
}

// Primal-weight update w <- exp(theta log(ratio) + (1 - theta) log(w)) (PDLP smoothing).  theta = 1 and
// theta = 0.5 have closed forms.  [r5] The general case is inlined too (DVH_PW_INLINE, default 1): as a call it
// bound the kernels' live registers to the call ABI at its call site -- inlined, the market days run 11.1 / 14.8 ms
// (market options / defaults) instead of 11.4 / 15.7 and config 3 168 instead of 174 ms
// (profiles/r05v_pw_inline.log).
#ifndef DVH_PW_INLINE
#define DVH_PW_INLINE 1
#endif
__device__ __forceinline__ double pw_update_general_i(double ratio, double w, double theta) {
  return exp(theta * log(ratio) + (1.0 - theta) * log(w));
}
__device__ __noinline__ double pw_update_general_o(double ratio, double w, double theta) {
  return pw_update_general_i(ratio, w, theta);
}
// INL = false: the general case out of line regardless (the band kernel's ICE form, whose 168-VGPR budget it strains)
template <bool INL = true>
__device__ __forceinline__ double pw_update(double ratio, double w, double theta) {
  if (theta == 1.0) return ratio;
  if (theta == 0.5) return sqrt(ratio * w);
  if constexpr (INL && DVH_PW_INLINE) return pw_update_general_i(ratio, w, theta);
  else return pw_update_general_o(ratio, w, theta);
}

// Makes an index opaque to the optimiser so that address arithmetic of cold (check-phase) code is not
// hoisted out of the iteration loop into long-lived VGPRs.
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ double opaque(double v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup release/acquire fence, which also
// waits for every outstanding global store of the wave to be acknowledged (s_waitcnt vmcnt(0)); in the PDHG
// loops global memory is only read back by the lane that wrote it, so that wait is pure latency.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Block reduction of NV doubles; red must hold (NW + 1) * NV doubles.  Result identical in all threads.
template <int B, int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* red) {
  constexpr int NW = B / kWave;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wid * NV + k] = v[k];
  }
  __syncthreads();
  if (tid < NV) {
    double s = 0.0;
    for (int w = 0; w < NW; ++w) s += red[w * NV + tid];
    red[NW * NV + tid] = s;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = red[NW * NV + k];
  __syncthreads();
}

// One-barrier variant: per-wave partials in red[wave*NV + k], one __syncthreads, then every lane adds the
// NW partials in wave order (identical, deterministic result in all lanes).  The caller must not reuse
// `red` before another barrier has passed (in the PDHG loop the next use is >= 2 barriers later).
template <int B, int NV, bool LDSB = false>
__device__ __forceinline__ void block_sum1(double (&v)[NV], double* red) {
  static_assert(NV <= kWave, "one lane per reduced value");
  constexpr int NW = B / kWave;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum_dpp(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wid * NV + k] = v[k];
  }
  if constexpr (LDSB)
    lds_barrier();
  else
    __syncthreads();
  // lane k adds value k over the waves (fixed order), then every value is broadcast from its lane
  double t = 0.0;
  if (lane < NV) {
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[w * NV + lane];
  }
  const int lo = __double2loint(t), hi = __double2hiint(t);
#pragma unroll
  for (int k = 0; k < NV; ++k)
    v[k] = __hiloint2double(__builtin_amdgcn_readlane(hi, k), __builtin_amdgcn_readlane(lo, k));
}

// Termination test of a KKT check (all quantities unscaled): relative primal / dual residual and gap <= eps,
// and, with eps_obj > 0, the objective-error estimate |pobj - dobj| + ||y||_2 ||r_p||_2 <= eps_obj (1 + |pobj|)
// (the gap plus the dual-weighted primal residual: what an infeasible candidate can gain on the optimum; it keeps
// every window's objective within 1e-5 of HiGHS where the KKT test alone let 1.08e-5 through).
// rdx: sum_j |r_d,j| |x_j|, what the dual objective can overstate the optimum by (p* >= dobj - sum_j
// |r_d,j| |x*_j|, with x in place of x*): a window whose dual residual sits on a large column (the demand charge's tau)
// otherwise stopped with its objective 1.6e-6 off (profiles/r04y_certify.json).  Every kernel applies it except the
// band ICE form (NRED = kNRed - 1 in dvh_band.hip: the term cost 6 % on config 5 through its check path's registers,
// DESIGN.md section 4), whose windows keep the round-3 test; both restatements (oracle/pdlp_ref.py,
// oracle/cpu_pdhg.cpp) apply it to every window, so an ICE window can end one check later there than on the GPU.
__device__ __forceinline__ bool kkt_done(const Opts& o, double pres, double dres, double gap, double pobj,
                                         double dobj, double rp2, double y2, double rdx = 0.0) {
  if (!(pres <= o.eps && dres <= o.eps && gap <= o.eps)) return false;
  return !(o.eps_obj > 0.0) || fabs(pobj - dobj) + sqrt(rp2 * y2) + rdx <= o.eps_obj * (1.0 + fabs(pobj));
}

// Predicted KKT gate (dvh_options.kkt_predict = P > 0): a due KKT check is skipped while the last check's worst
// ratio max(pres, dres, gap) / eps, scaled by the fixed-point residual's decrease since then (r / r_then), exceeds P,
// at most kKktMaxSkip due checks in a row.  Only the timing of the termination test changes, not the iterates.
constexpr int kKktMaxSkip = 4;
struct KktGate {
  double q = -1.0, r = 0.0;  // the last KKT check's worst ratio to eps and fixed-point residual (q < 0: none yet)
  int skip = 0;              // due checks skipped since
  __device__ void note(double pres, double dres, double gap, double eps, double rr) {
    q = fmax(fmax(pres, dres), gap) / eps;
    r = rr;
    skip = 0;
  }
};
__device__ __forceinline__ bool kkt_gate_skip(const Opts& o, const KktGate& g, double r) {
  return g.q >= 0.0 && g.skip < kKktMaxSkip && g.q * r > (double)o.kkt_predict * g.r;
}

struct WinOff {
  int n, m, meq, nnz;
  int64_t row, nz, on, om;     // global offsets (inputs / outputs)
  int64_t wn, wm, wz, wtr;     // chunk-relative workspace offsets
};

__device__ __forceinline__ WinOff win_offsets(const Batch& b, const Chunk& ch, int k) {
  const int64_t* d = b.desc + 8 * (int64_t)k;
  WinOff o;
  o.n = (int)d[0];
  o.m = (int)d[1];
  o.meq = (int)d[2];
  o.nnz = (int)d[3];
  o.row = d[4];
  o.nz = d[5];
  o.on = d[6];
  o.om = d[7];
  o.wn = o.on - ch.base_n;
  o.wm = o.om - ch.base_m;
  o.wz = o.nz - ch.base_nz;
  o.wtr = o.wn + (k - ch.first);
  return o;
}

// A wave-uniform 64-bit value made scalar (v_readfirstlane of both halves), and a window's offsets likewise: read with
// vector loads (the kernels write global memory, so the compiler does not treat the descriptors as constant), they and
// every address formed from them would sit in VGPR pairs.
__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(unsigned long long)v);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)((unsigned long long)v >> 32));
  return (int64_t)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ WinOff uniform_win(WinOff o) {
  o.n = __builtin_amdgcn_readfirstlane(o.n);
  o.m = __builtin_amdgcn_readfirstlane(o.m);
  o.meq = __builtin_amdgcn_readfirstlane(o.meq);
  o.nnz = __builtin_amdgcn_readfirstlane(o.nnz);
  o.row = uniform_i64(o.row);
  o.nz = uniform_i64(o.nz);
  o.on = uniform_i64(o.on);
  o.om = uniform_i64(o.om);
  o.wn = uniform_i64(o.wn);
  o.wm = uniform_i64(o.wm);
  o.wz = uniform_i64(o.wz);
  o.wtr = uniform_i64(o.wtr);
  return o;
}

// LDS f64 load / store at an absolute LDS byte address (precomputed once in a VGPR, so a gather is a single
// ds_read_b64 with no address arithmetic in the loop).
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) unsigned char lds_u8;
__device__ __forceinline__ int lds_addr(const void* p) {
  return (int)(size_t)(lds_u8*)(p);
}
__device__ __forceinline__ double lds_ld(int a) { return *(lds_f64*)(size_t)(unsigned)a; }
__device__ __forceinline__ void lds_st(int a, double v) { *(lds_f64*)(size_t)(unsigned)a = v; }
// Plain v_max_f64 / v_min_f64: the operands are finite or +-inf by construction (no NaN inputs), so the
// IEEE-mode canonicalisation the compiler would insert before every use of a loop-invariant bound is dead.
__device__ __forceinline__ double vmax(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double uniform(double v) {
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                          __builtin_amdgcn_readfirstlane(__double2loint(v)));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}

}  // namespace
}  // namespace dvh

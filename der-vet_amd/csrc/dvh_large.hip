// dvh_large.hip -- grid-wide restarted Halpern PDHG for one window that is too large for a workgroup.
//
// BASELINE config 3 is a single annual 5-minute window (T = 105,120 steps: n = 3T, m = T + 1, or with monthly
// DCM n = 3T + 12, m = 2T + 1).  It replaces the same storagevet Scenario.solve_optimization call
// (dervet/MicrogridScenario.py:319) as the batched kernels, for windows with n or m above kSmallMax.
//
// The arithmetic is the one of oracle/pdlp_ref.py (Ruiz + Pock-Chambolle scaling, power-iteration step,
// reflected Halpern PDHG, fixed-point restarts every check_every iterations, unscaled relative KKT
// termination every kkt_every checks).  The mapping onto the GPU:
//   * one thread per column (primal half-step) or per row (dual half-step), column-major ELL slices for
//     rows / columns with <= kLgLong entries (coalesced: entry e of row i at e * m + i);
//   * every longer row / column (the DCM tau columns: one entry per step of the month) gets a workgroup of
//     its own inside the same launch, so a half-step is exactly one kernel;
//   * restart / termination decisions are made on the device by a one-workgroup check kernel from
//     per-workgroup partial sums (fixed summation order -> bitwise reproducible), and applied by an
//     element-wise restart kernel;
//   * one check period (check_every iterations: 2 * check_every half-step kernels + 2 KKT kernels + check +
//     restart) is captured once as a hipGraph and replayed; the host polls the status one replay behind.
// Kernel boundaries (~1.5 us) are cheaper than grid barriers (~4-5 us) on MI355X at this grid size, which
// is why the half-steps are separate launches rather than one persistent kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "dvh_internal.h"

namespace dvh {
namespace {

constexpr int LB = 256;         // threads per workgroup
constexpr int kLgLong = 32;     // rows / columns longer than this get their own workgroup
constexpr int kPart = 8;        // partial sums per workgroup
constexpr int kOptimal = 0, kIterLimit = 3, kNumerical = 4;

struct LgState {
  double eta, w, tau, sigma;
  double r0, rprev;                  // < 0: unset
  double pres, dres, gap, pobj;      // last KKT evaluation (relative residuals, primal objective)
  double pscale, sig;                // power iteration: 1 / |v|, sqrt(|K'K v|)
  double ncs, nqs, nc, nq;           // ||c_s||, ||q_s||, ||c||, ||q||
  int it, kin, status, restart;
};

struct LgArgs {
  int n, m, meq;
  int wr, wc;      // ELL widths of K rows / K^T rows (columns of K)
  int nlr, nlc;    // long rows / long columns
  int nbr, nbc;    // short-element workgroups over rows / columns
  // ELL (scaled values filled on device) and long lists in CSR form
  const int32_t* ki; const int32_t* kpos; double* kv;     // [wr * m]
  const int32_t* ti; const int32_t* tpos; double* tv;     // [wc * n]
  const int32_t* lr; const int32_t* lrp; const int32_t* lri; const int32_t* lrpos; double* lrv;
  const int32_t* lc; const int32_t* lcp; const int32_t* lci; const int32_t* lcpos; double* lcv;
  const uint8_t* rlong; const uint8_t* clong;
  // full transpose (setup passes): Tp[n+1], Ti (row ids), Tpos (K entry of each K^T slot)
  const int32_t* Tp; const int32_t* Ti; const int32_t* Tpos;
  // window inputs (unscaled)
  const int32_t* Kp; const int32_t* Kc; const double* Kv;
  const double* c; const double* q; const double* l; const double* u; double c0;
  // scaled data
  double *dr, *dc, *cs, *ls, *us, *qs, *tmpr, *tmpc;
  // iterates
  double *x, *xa, *xo, *xb, *y, *ya, *yo;
  double* part;          // [(nbc + nlc + nbr + nlr) * kPart]
  const double* hinv;
  LgState* st;
  double eps, rho, b_suff, b_nec, b_art, theta, step_safety, eps_obj;
  int chk, kkt_every, max_iters;
  int warm;              // 1: start from the unscaled x / y already in the output buffers (dvh_options.warm_start)
  // outputs
  double* ox; double* oy; double* ostats; int32_t* oist;
};

__device__ __forceinline__ double lg_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Deterministic workgroup sum of NV values; result valid in thread 0.
template <int NV>
__device__ __forceinline__ void lg_block_sum(double (&v)[NV]) {
  __shared__ double red[NV * (LB / 64)];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = lg_wave_sum(v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wid * NV + k] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = 0.0;
      for (int t = 0; t < LB / 64; ++t) s += red[t * NV + k];
      v[k] = s;
    }
  }
}

__device__ __forceinline__ double halpern_cb(const LgArgs& a, int kin) {
  return kin < kHalpernTab ? a.hinv[kin] : 1.0 / (kin + 2.0);
}

// ------------------------------------------------------------------------------------------------
// setup
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(LB) void lg_ones(LgArgs a) {
  const int t = blockIdx.x * LB + threadIdx.x;
  if (t < a.n) a.dc[t] = 1.0;
  if (t < a.m) a.dr[t] = 1.0;
}

// One Ruiz (max) or Pock-Chambolle (sum) pass: row factors into tmpr, column factors into tmpc.
template <bool MAXR>
__global__ __launch_bounds__(LB) void lg_scale_pass(LgArgs a) {
  const int t = blockIdx.x * LB + threadIdx.x;
  if (t < a.m) {
    double acc = 0.0;
    const double d = a.dr[t];
    for (int p = a.Kp[t]; p < a.Kp[t + 1]; ++p) {
      const double v = fabs(a.Kv[p]) * d * a.dc[a.Kc[p]];
      acc = MAXR ? fmax(acc, v) : acc + v;
    }
    a.tmpr[t] = acc > 0.0 ? 1.0 / sqrt(acc) : 1.0;
  }
  if (t < a.n) {
    double acc = 0.0;
    const double d = a.dc[t];
    for (int p = a.Tp[t]; p < a.Tp[t + 1]; ++p) {
      const double v = fabs(a.Kv[a.Tpos[p]]) * d * a.dr[a.Ti[p]];
      acc = MAXR ? fmax(acc, v) : acc + v;
    }
    a.tmpc[t] = acc > 0.0 ? 1.0 / sqrt(acc) : 1.0;
  }
}

__global__ __launch_bounds__(LB) void lg_scale_apply(LgArgs a) {
  const int t = blockIdx.x * LB + threadIdx.x;
  if (t < a.n) a.dc[t] *= a.tmpc[t];
  if (t < a.m) a.dr[t] *= a.tmpr[t];
}

// Scaled matrix values into the ELL slices and long lists; scaled vectors; norm partials.
__global__ __launch_bounds__(LB) void lg_fill(LgArgs a) {
  const int t = blockIdx.x * LB + threadIdx.x;
  double nv[4] = {0.0, 0.0, 0.0, 0.0};
  if (t < a.m) {
    const double d = a.dr[t];
    for (int e = 0; e < a.wr; ++e) {
      const size_t s = (size_t)e * a.m + t;
      const int p = a.kpos[s];
      a.kv[s] = p >= 0 ? a.Kv[p] * d * a.dc[a.ki[s]] : 0.0;
    }
    const double qi = a.q[t];
    a.qs[t] = qi * d;
    nv[1] = qi * d * qi * d;
    nv[3] = qi * qi;
  }
  if (t < a.n) {
    const double d = a.dc[t];
    for (int e = 0; e < a.wc; ++e) {
      const size_t s = (size_t)e * a.n + t;
      const int p = a.tpos[s];
      a.tv[s] = p >= 0 ? a.Kv[p] * d * a.dr[a.ti[s]] : 0.0;
    }
    const double cj = a.c[t];
    a.cs[t] = cj * d;
    a.ls[t] = a.l[t] / d;
    a.us[t] = a.u[t] / d;
    nv[0] = cj * d * cj * d;
    nv[2] = cj * cj;
  }
  // long lists (a few thousand entries each; strided over the whole grid)
  for (int L = 0; L < a.nlr; ++L) {
    const int i = a.lr[L];
    for (int p = a.lrp[L] + t; p < a.lrp[L + 1]; p += gridDim.x * LB)
      a.lrv[p] = a.Kv[a.lrpos[p]] * a.dr[i] * a.dc[a.lri[p]];
  }
  for (int L = 0; L < a.nlc; ++L) {
    const int j = a.lc[L];
    for (int p = a.lcp[L] + t; p < a.lcp[L + 1]; p += gridDim.x * LB)
      a.lcv[p] = a.Kv[a.lcpos[p]] * a.dc[j] * a.dr[a.lci[p]];
  }
  lg_block_sum<4>(nv);
  if (threadIdx.x == 0)
    for (int k = 0; k < 4; ++k) a.part[(size_t)blockIdx.x * kPart + k] = nv[k];
}

// Sum of the first NV partials over nblk workgroups (one workgroup of 1024 threads, fixed order).
template <int NV>
__device__ void lg_reduce_parts(const double* part, int first, int nblk, int off, double (&out)[NV]) {
  __shared__ double red[NV * 16];
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += part[(size_t)(first + b) * kPart + off + k];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = lg_wave_sum(v[k]);
  __syncthreads();
  if (lane == 0)
    for (int k = 0; k < NV; ++k) red[wid * NV + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = 0.0;
    for (int t = 0; t < (int)(blockDim.x >> 6); ++t) s += red[t * NV + k];
    out[k] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void lg_setup_norms(LgArgs a, int nblk) {
  double s[4];
  lg_reduce_parts<4>(a.part, 0, nblk, 0, s);
  if (threadIdx.x == 0) {
    LgState* st = a.st;
    st->ncs = sqrt(s[0]);
    st->nqs = sqrt(s[1]);
    st->nc = sqrt(s[2]);
    st->nq = sqrt(s[3]);
    st->pscale = 1.0;
    st->sig = 1.0;
  }
}

// power iteration on Kt'Kt: rows  w = Kt (pscale * v)
__global__ __launch_bounds__(LB) void lg_pow_rows(LgArgs a, const double* v, double* wv) {
  const double s = a.st->pscale;
  if ((int)blockIdx.x < a.nbr) {
    const int i = blockIdx.x * LB + threadIdx.x;
    if (i < a.m && !a.rlong[i]) {
      double acc = 0.0;
      for (int e = 0; e < a.wr; ++e) acc += a.kv[(size_t)e * a.m + i] * v[a.ki[(size_t)e * a.m + i]];
      wv[i] = s * acc;
    }
  } else {
    const int L = blockIdx.x - a.nbr;
    double acc[1] = {0.0};
    for (int p = a.lrp[L] + threadIdx.x; p < a.lrp[L + 1]; p += LB) acc[0] += a.lrv[p] * v[a.lri[p]];
    lg_block_sum<1>(acc);
    if (threadIdx.x == 0) wv[a.lr[L]] = s * acc[0];
  }
}

// power iteration: columns  v = Kt' w, partial |v|^2
__global__ __launch_bounds__(LB) void lg_pow_cols(LgArgs a, const double* wv, double* v) {
  double nv[1] = {0.0};
  if ((int)blockIdx.x < a.nbc) {
    const int j = blockIdx.x * LB + threadIdx.x;
    if (j < a.n && !a.clong[j]) {
      double acc = 0.0;
      for (int e = 0; e < a.wc; ++e) acc += a.tv[(size_t)e * a.n + j] * wv[a.ti[(size_t)e * a.n + j]];
      v[j] = acc;
      nv[0] = acc * acc;
    }
    lg_block_sum<1>(nv);
  } else {
    const int L = blockIdx.x - a.nbc;
    double acc[1] = {0.0};
    for (int p = a.lcp[L] + threadIdx.x; p < a.lcp[L + 1]; p += LB) acc[0] += a.lcv[p] * wv[a.lci[p]];
    lg_block_sum<1>(acc);
    if (threadIdx.x == 0) {
      v[a.lc[L]] = acc[0];
      nv[0] = acc[0] * acc[0];
    }
  }
  if (threadIdx.x == 0) a.part[(size_t)blockIdx.x * kPart] = nv[0];
}

__global__ __launch_bounds__(1024) void lg_pow_norm(LgArgs a, int nblk) {
  double s[1];
  lg_reduce_parts<1>(a.part, 0, nblk, 0, s);
  if (threadIdx.x == 0) {
    const double nv = sqrt(s[0]);
    if (nv > 0.0) {
      a.st->sig = sqrt(nv);
      a.st->pscale = 1.0 / nv;
    }
  }
}

__global__ __launch_bounds__(LB) void lg_start(LgArgs a) {
  const int t = blockIdx.x * LB + threadIdx.x;
  if (t < a.n) {
    const double x0 = fmin(fmax(a.warm ? a.ox[t] / a.dc[t] : 0.0, a.ls[t]), a.us[t]);
    a.x[t] = x0;
    a.xa[t] = x0;
    a.xo[t] = x0;
    a.xb[t] = x0;
  }
  if (t < a.m) {
    double y0 = a.warm ? a.oy[t] / a.dr[t] : 0.0;
    if (t >= a.meq) y0 = fmax(y0, 0.0);  // >= rows: dual feasibility of the start
    a.y[t] = y0;
    a.ya[t] = y0;
    a.yo[t] = y0;
  }
  if (t == 0) {
    LgState* st = a.st;
    st->eta = a.step_safety / st->sig;
    st->w = (st->ncs > 1e-10 && st->nqs > 1e-10) ? st->ncs / st->nqs : 1.0;
    st->tau = st->eta / st->w;
    st->sigma = st->eta * st->w;
    st->r0 = -1.0;
    st->rprev = -1.0;
    st->it = 0;
    st->kin = 0;
    st->status = -1;
    st->restart = 0;
    st->pres = st->dres = st->gap = INFINITY;
    st->pobj = 0.0;
  }
}

// ------------------------------------------------------------------------------------------------
// iteration
// ------------------------------------------------------------------------------------------------
template <bool CHECK>
__device__ __forceinline__ void x_update(const LgArgs& a, int j, double kty, double tau, double ca, double cb,
                                         double& mv0, double& mv1) {
  const double xv = a.x[j];
  const double p1 = fmin(fmax(xv - tau * (a.cs[j] - kty), a.ls[j]), a.us[j]);
  const double xb = 2.0 * p1 - xv;
  a.xb[j] = xb;
  const double xan = a.xa[j];
  if (CHECK) {
    const double d = xv - p1, da = p1 - xan;
    mv0 += d * d;
    mv1 += da * da;
    a.xo[j] = p1;
  }
  a.x[j] = ca * ((1.0 + a.rho) * p1 - a.rho * xv) + cb * xan;
}

template <bool CHECK>
__global__ __launch_bounds__(LB) void lg_primal(LgArgs a, int i) {
  const LgState* st = a.st;
  if (st->status >= 0) return;
  const int kin = st->kin + i;
  const double cb = halpern_cb(a, kin), ca = 1.0 - cb;
  const double tau = st->tau;
  double mv[2] = {0.0, 0.0};
  if ((int)blockIdx.x < a.nbc) {
    const int j = blockIdx.x * LB + threadIdx.x;
    if (j < a.n && !a.clong[j]) {
      double kty = 0.0;
      for (int e = 0; e < a.wc; ++e) kty += a.tv[(size_t)e * a.n + j] * a.y[a.ti[(size_t)e * a.n + j]];
      x_update<CHECK>(a, j, kty, tau, ca, cb, mv[0], mv[1]);
    }
    if (CHECK) lg_block_sum<2>(mv);
  } else {
    const int L = blockIdx.x - a.nbc;
    double acc[1] = {0.0};
    for (int p = a.lcp[L] + threadIdx.x; p < a.lcp[L + 1]; p += LB) acc[0] += a.lcv[p] * a.y[a.lci[p]];
    lg_block_sum<1>(acc);
    if (threadIdx.x == 0) x_update<CHECK>(a, a.lc[L], acc[0], tau, ca, cb, mv[0], mv[1]);
  }
  if (CHECK && threadIdx.x == 0) {
    a.part[(size_t)blockIdx.x * kPart + 0] = mv[0];
    a.part[(size_t)blockIdx.x * kPart + 1] = mv[1];
  }
}

template <bool CHECK>
__device__ __forceinline__ void y_update(const LgArgs& a, int r, double kx, double sigma, double ca, double cb,
                                         double& mv2, double& mv3) {
  const double yv = a.y[r];
  double yp = yv + sigma * (a.qs[r] - kx);
  if (r >= a.meq) yp = fmax(yp, 0.0);
  const double yan = a.ya[r];
  if (CHECK) {
    const double d = yv - yp, da = yp - yan;
    mv2 += d * d;
    mv3 += da * da;
    a.yo[r] = yp;
  }
  a.y[r] = ca * ((1.0 + a.rho) * yp - a.rho * yv) + cb * yan;
}

template <bool CHECK>
__global__ __launch_bounds__(LB) void lg_dual(LgArgs a, int i) {
  const LgState* st = a.st;
  if (st->status >= 0) return;
  const int kin = st->kin + i;
  const double cb = halpern_cb(a, kin), ca = 1.0 - cb;
  const double sigma = st->sigma;
  const int pb = a.nbc + a.nlc + blockIdx.x;  // partial slot (row workgroups after the column ones)
  double mv[2] = {0.0, 0.0};
  if ((int)blockIdx.x < a.nbr) {
    const int r = blockIdx.x * LB + threadIdx.x;
    if (r < a.m && !a.rlong[r]) {
      double kx = 0.0;
      for (int e = 0; e < a.wr; ++e) kx += a.kv[(size_t)e * a.m + r] * a.xb[a.ki[(size_t)e * a.m + r]];
      y_update<CHECK>(a, r, kx, sigma, ca, cb, mv[0], mv[1]);
    }
    if (CHECK) lg_block_sum<2>(mv);
  } else {
    const int L = blockIdx.x - a.nbr;
    double acc[1] = {0.0};
    for (int p = a.lrp[L] + threadIdx.x; p < a.lrp[L + 1]; p += LB) acc[0] += a.lrv[p] * a.xb[a.lri[p]];
    lg_block_sum<1>(acc);
    if (threadIdx.x == 0) y_update<CHECK>(a, a.lr[L], acc[0], sigma, ca, cb, mv[0], mv[1]);
  }
  if (CHECK && threadIdx.x == 0) {
    a.part[(size_t)pb * kPart + 0] = mv[0];
    a.part[(size_t)pb * kPart + 1] = mv[1];
  }
}

__device__ __forceinline__ bool is_kkt_check(const LgArgs& a, const LgState* st) {
  const int after = st->it + a.chk;
  return (after / a.chk) % a.kkt_every == 0 || after + a.chk > a.max_iters;
}

// KKT rows: |(q - K x)_+|^2 and q'y of the candidate (xo, yo), unscaled.
__global__ __launch_bounds__(LB) void lg_kkt_rows(LgArgs a) {
  const LgState* st = a.st;
  if (st->status >= 0 || !is_kkt_check(a, st)) return;
  const int pb = a.nbc + a.nlc + blockIdx.x;
  double v[3] = {0.0, 0.0, 0.0};
  auto acc = [&](int r, double kxs) {
    double res = a.q[r] - kxs / a.dr[r];
    if (r >= a.meq) res = fmax(res, 0.0);
    const double yu = a.dr[r] * a.yo[r];
    v[0] += res * res;
    v[1] += a.q[r] * yu;
    v[2] += yu * yu;
  };
  if ((int)blockIdx.x < a.nbr) {
    const int r = blockIdx.x * LB + threadIdx.x;
    if (r < a.m && !a.rlong[r]) {
      double kx = 0.0;
      for (int e = 0; e < a.wr; ++e) kx += a.kv[(size_t)e * a.m + r] * a.xo[a.ki[(size_t)e * a.m + r]];
      acc(r, kx);
    }
    lg_block_sum<3>(v);
  } else {
    const int L = blockIdx.x - a.nbr;
    double s[1] = {0.0};
    for (int p = a.lrp[L] + threadIdx.x; p < a.lrp[L + 1]; p += LB) s[0] += a.lrv[p] * a.xo[a.lri[p]];
    lg_block_sum<1>(s);
    if (threadIdx.x == 0) acc(a.lr[L], s[0]);
  }
  if (threadIdx.x == 0) {
    a.part[(size_t)pb * kPart + 2] = v[0];
    a.part[(size_t)pb * kPart + 3] = v[1];
    a.part[(size_t)pb * kPart + 4] = v[2];
  }
}

// KKT columns: reduced-cost residual |rc - lambda|^2, c'x, bound part of the dual objective, sum |r_d| |x| (the objective
// gate's dual-residual term, csrc/dvh_device.h kkt_done).
__global__ __launch_bounds__(LB) void lg_kkt_cols(LgArgs a) {
  const LgState* st = a.st;
  if (st->status >= 0 || !is_kkt_check(a, st)) return;
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  auto acc = [&](int j, double ktys) {
    const double rc = a.c[j] - ktys / a.dc[j];
    const double lo = a.l[j], hi = a.u[j];
    const bool fl = lo > -INFINITY, fu = hi < INFINITY;
    const double lam = (fl && fu) ? rc : fl ? fmax(rc, 0.0) : fu ? fmin(rc, 0.0) : 0.0;
    const double rd = rc - lam;
    v[0] += rd * rd;
    v[1] += a.c[j] * (a.dc[j] * a.xo[j]);
    v[2] += (fl ? lo * fmax(lam, 0.0) : 0.0) + (fu ? hi * fmin(lam, 0.0) : 0.0);
    v[3] += fabs(rd) * fabs(a.dc[j] * a.xo[j]);
  };
  if ((int)blockIdx.x < a.nbc) {
    const int j = blockIdx.x * LB + threadIdx.x;
    if (j < a.n && !a.clong[j]) {
      double kty = 0.0;
      for (int e = 0; e < a.wc; ++e) kty += a.tv[(size_t)e * a.n + j] * a.yo[a.ti[(size_t)e * a.n + j]];
      acc(j, kty);
    }
    lg_block_sum<4>(v);
  } else {
    const int L = blockIdx.x - a.nbc;
    double s[1] = {0.0};
    for (int p = a.lcp[L] + threadIdx.x; p < a.lcp[L + 1]; p += LB) s[0] += a.lcv[p] * a.yo[a.lci[p]];
    lg_block_sum<1>(s);
    if (threadIdx.x == 0) acc(a.lc[L], s[0]);
  }
  if (threadIdx.x == 0) {
    a.part[(size_t)blockIdx.x * kPart + 2] = v[0];
    a.part[(size_t)blockIdx.x * kPart + 3] = v[1];
    a.part[(size_t)blockIdx.x * kPart + 4] = v[2];
    a.part[(size_t)blockIdx.x * kPart + 5] = v[3];
  }
}

// Restart / termination decision of one check (oracle/pdlp_ref.py solve(), the `it % check_every == 0` branch).
__global__ __launch_bounds__(1024) void lg_check(LgArgs a) {
  LgState* st = a.st;
  if (st->status >= 0) return;
  const int ncb = a.nbc + a.nlc, nrb = a.nbr + a.nlr;
  const bool kkt = is_kkt_check(a, st);
  double cm[2], rm[2], ck[4] = {0.0, 0.0, 0.0, 0.0}, rk[3] = {0.0, 0.0, 0.0};
  lg_reduce_parts<2>(a.part, 0, ncb, 0, cm);
  lg_reduce_parts<2>(a.part, ncb, nrb, 0, rm);
  if (kkt) {
    lg_reduce_parts<4>(a.part, 0, ncb, 2, ck);
    lg_reduce_parts<3>(a.part, ncb, nrb, 2, rk);
  }
  if (threadIdx.x != 0) return;
  const int after = st->it + a.chk;
  const double w = st->w;
  const double r = sqrt(w * cm[0] + rm[0] / w);
  st->restart = 0;
  st->it = after;
  if (kkt) {
    const double pobj = ck[1] + a.c0;
    const double dobj = rk[1] + ck[2] + a.c0;
    st->pres = sqrt(rk[0]) / (1.0 + st->nq);
    st->dres = sqrt(ck[0]) / (1.0 + st->nc);
    st->gap = fabs(pobj - dobj) / (1.0 + fabs(pobj) + fabs(dobj));
    st->pobj = pobj;
    const bool obj_ok =
        !(a.eps_obj > 0.0) || fabs(pobj - dobj) + sqrt(rk[0] * rk[2]) + ck[3] <= a.eps_obj * (1.0 + fabs(pobj));
    if (st->pres <= a.eps && st->dres <= a.eps && st->gap <= a.eps && obj_ok) {
      st->status = kOptimal;
      return;
    }
    if (!isfinite(st->pres) || !isfinite(st->dres) || !isfinite(st->gap)) {
      st->status = kNumerical;
      return;
    }
  }
  if (!isfinite(r)) {
    st->status = kNumerical;
    return;
  }
  if (st->r0 < 0.0) st->r0 = r;
  const int kcheck = st->kin + a.chk - 1;  // inner Halpern count of the check iteration
  const bool restart = (r <= a.b_suff * st->r0) || (r <= a.b_nec * st->r0 && st->rprev >= 0.0 && r > st->rprev) ||
                       (kcheck + 1 >= a.b_art * after);
  if (restart) {
    const double ddx = sqrt(cm[1]), ddy = sqrt(rm[1]);
    if (ddx > 1e-10 && ddy > 1e-10) {
      const double wn = a.theta == 1.0 ? ddy / ddx : exp(a.theta * log(ddy / ddx) + (1.0 - a.theta) * log(w));
      st->w = wn;
      st->tau = st->eta / wn;
      st->sigma = st->eta * wn;
    }
    st->restart = 1;
    st->kin = 0;
    st->r0 = r;
    st->rprev = -1.0;
  } else {
    st->rprev = r;
    st->kin += a.chk;
  }
  if (after + a.chk > a.max_iters) st->status = kIterLimit;
}

__global__ __launch_bounds__(LB) void lg_restart(LgArgs a) {
  const LgState* st = a.st;
  if (!st->restart || st->status >= 0) return;
  const int t = blockIdx.x * LB + threadIdx.x;
  if (t < a.n) {
    const double v = a.xo[t];
    a.x[t] = v;
    a.xa[t] = v;
  }
  if (t < a.m) {
    const double v = a.yo[t];
    a.y[t] = v;
    a.ya[t] = v;
  }
}

__global__ __launch_bounds__(LB) void lg_finish(LgArgs a) {
  const LgState* st = a.st;
  const int t = blockIdx.x * LB + threadIdx.x;
  if (t < a.n) a.ox[t] = a.dc[t] * a.xo[t];
  if (t < a.m) a.oy[t] = a.dr[t] * a.yo[t];
  if (t == 0) {
    a.ostats[0] = st->pobj;
    a.ostats[1] = st->pres;
    a.ostats[2] = st->dres;
    a.ostats[3] = st->gap;
    a.oist[0] = st->status < 0 ? kIterLimit : st->status;
    a.oist[1] = st->status == kIterLimit ? a.max_iters : st->it;
  }
}

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t want) {
    want = std::max<size_t>(want, 256);
    if (want <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) bytes = want;
    return e;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

}  // namespace

struct LargeSolver {
  Buf ints, dbls, st;
  int32_t* pinned_status = nullptr;
  hipStream_t cap = nullptr;  // graph-capture stream (capture never executes work)
  hipEvent_t poll[2] = {nullptr, nullptr};
  hipEvent_t tev[3] = {nullptr, nullptr, nullptr};  // setup / PDHG timing brackets, reused by every solve
  ~LargeSolver() {
    for (Buf* b : {&ints, &dbls, &st})
      if (b->p) (void)hipFree(b->p);
    if (pinned_status) (void)hipHostFree(pinned_status);
    for (hipEvent_t e : poll)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : tev)
      if (e) (void)hipEventDestroy(e);
    if (cap) (void)hipStreamDestroy(cap);
  }
};

namespace {
// one check period's graph and its executable, destroyed on every return path
struct GraphGuard {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  ~GraphGuard() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
  }
};
}  // namespace

LargeSolver* large_create() { return new LargeSolver(); }
void large_destroy(LargeSolver* ls) { delete ls; }

#define LG_TRY(call)                           \
  do {                                         \
    hipError_t e_ = (call);                    \
    if (e_ != hipSuccess) {                    \
      if (err) *err = std::string(#call) + ": " + hipGetErrorString(e_); \
      return e_;                               \
    }                                          \
  } while (0)

hipError_t large_solve(LargeSolver* ls, const Batch& b, int k, const int64_t* d, const Opts& o, const double* hinv,
                       hipStream_t s, std::string* err, float* setup_ms, float* pdhg_ms) {
  const int n = (int)d[0], m = (int)d[1], meq = (int)d[2], nnz = (int)d[3];
  const int64_t orow = d[4], onz = d[5], on = d[6], om = d[7];
  // ---- pattern on the host: transpose, long lists, ELL index slices
  std::vector<int32_t> Kp(m + 1), Kc(std::max(nnz, 1));
  LG_TRY(hipMemcpyAsync(Kp.data(), b.indptr + orow, sizeof(int32_t) * (m + 1), hipMemcpyDeviceToHost, s));
  if (nnz) LG_TRY(hipMemcpyAsync(Kc.data(), b.indices + onz, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost, s));
  LG_TRY(hipStreamSynchronize(s));
  std::vector<int32_t> Tp(n + 1, 0), Ti(std::max(nnz, 1)), Tpos(std::max(nnz, 1));
  for (int p = 0; p < nnz; ++p) Tp[Kc[p] + 1]++;
  for (int j = 0; j < n; ++j) Tp[j + 1] += Tp[j];
  {
    std::vector<int32_t> cur(Tp.begin(), Tp.end() - 1);
    for (int i = 0; i < m; ++i)
      for (int p = Kp[i]; p < Kp[i + 1]; ++p) {
        const int q = cur[Kc[p]]++;
        Ti[q] = i;
        Tpos[q] = p;
      }
  }
  int wr = 0, wc = 0;
  std::vector<int32_t> lr, lrp{0}, lri, lrpos, lc, lcp{0}, lci, lcpos;
  std::vector<uint8_t> rlong(m, 0), clong(n, 0);
  for (int i = 0; i < m; ++i) {
    const int len = Kp[i + 1] - Kp[i];
    if (len > kLgLong) {
      rlong[i] = 1;
      lr.push_back(i);
      for (int p = Kp[i]; p < Kp[i + 1]; ++p) {
        lri.push_back(Kc[p]);
        lrpos.push_back(p);
      }
      lrp.push_back((int)lri.size());
    } else {
      wr = std::max(wr, len);
    }
  }
  for (int j = 0; j < n; ++j) {
    const int len = Tp[j + 1] - Tp[j];
    if (len > kLgLong) {
      clong[j] = 1;
      lc.push_back(j);
      for (int p = Tp[j]; p < Tp[j + 1]; ++p) {
        lci.push_back(Ti[p]);
        lcpos.push_back(Tpos[p]);
      }
      lcp.push_back((int)lci.size());
    } else {
      wc = std::max(wc, len);
    }
  }
  std::vector<int32_t> ki((size_t)wr * m, 0), kpos((size_t)wr * m, -1), ti((size_t)wc * n, 0), tpos((size_t)wc * n, -1);
  for (int i = 0; i < m; ++i) {
    if (rlong[i]) continue;
    for (int p = Kp[i], e = 0; p < Kp[i + 1]; ++p, ++e) {
      ki[(size_t)e * m + i] = Kc[p];
      kpos[(size_t)e * m + i] = p;
    }
  }
  for (int j = 0; j < n; ++j) {
    if (clong[j]) continue;
    for (int p = Tp[j], e = 0; p < Tp[j + 1]; ++p, ++e) {
      ti[(size_t)e * n + j] = Ti[p];
      tpos[(size_t)e * n + j] = Tpos[p];
    }
  }
  const int nlr = (int)lr.size(), nlc = (int)lc.size();
  const int nbr = (m + LB - 1) / LB, nbc = (n + LB - 1) / LB;
  const int nbe = std::max(nbr, nbc);  // element-wise grids over max(n, m)
  const int nparts = std::max(nbc + nlc + nbr + nlr, nbe);

  // ---- device buffers: one int arena, one double arena
  std::vector<std::pair<const std::vector<int32_t>*, size_t>> iv;
  size_t ioff = 0;
  auto iput = [&](const std::vector<int32_t>& v) {
    const size_t o = ioff;
    iv.push_back({&v, o});
    ioff += (v.size() + 63) & ~size_t(63);
    return o;
  };
  const size_t o_ki = iput(ki), o_kpos = iput(kpos), o_ti = iput(ti), o_tpos = iput(tpos), o_lr = iput(lr),
               o_lrp = iput(lrp), o_lri = iput(lri), o_lrpos = iput(lrpos), o_lc = iput(lc), o_lcp = iput(lcp),
               o_lci = iput(lci), o_lcpos = iput(lcpos), o_Tp = iput(Tp), o_Ti = iput(Ti), o_Tpos = iput(Tpos);
  const size_t o_flags = ioff;
  ioff += ((size_t)m + n + 255) / 4 + 64;
  LG_TRY(ls->ints.ensure(sizeof(int32_t) * ioff));
  int32_t* ib = ls->ints.as<int32_t>();
  for (auto& pr : iv)
    if (!pr.first->empty())
      LG_TRY(hipMemcpyAsync(ib + pr.second, pr.first->data(), sizeof(int32_t) * pr.first->size(),
                            hipMemcpyHostToDevice, s));
  uint8_t* fl = reinterpret_cast<uint8_t*>(ib + o_flags);
  if (m) LG_TRY(hipMemcpyAsync(fl, rlong.data(), m, hipMemcpyHostToDevice, s));
  if (n) LG_TRY(hipMemcpyAsync(fl + m, clong.data(), n, hipMemcpyHostToDevice, s));

  size_t doff = 0;
  auto dput = [&](size_t cnt) {
    const size_t o = doff;
    doff += (std::max<size_t>(cnt, 1) + 31) & ~size_t(31);
    return o;
  };
  const size_t o_kv = dput((size_t)wr * m), o_tv = dput((size_t)wc * n), o_lrv = dput(lri.size()),
               o_lcv = dput(lci.size()), o_dr = dput(m), o_dc = dput(n), o_cs = dput(n), o_ls = dput(n),
               o_us = dput(n), o_qs = dput(m), o_tmpr = dput(m), o_tmpc = dput(n), o_x = dput(n), o_xa = dput(n),
               o_xo = dput(n), o_xb = dput(n), o_y = dput(m), o_ya = dput(m), o_yo = dput(m),
               o_part = dput((size_t)nparts * kPart);
  LG_TRY(ls->dbls.ensure(sizeof(double) * doff));
  LG_TRY(ls->st.ensure(sizeof(LgState)));
  if (!ls->pinned_status) LG_TRY(hipHostMalloc(reinterpret_cast<void**>(&ls->pinned_status), 2 * sizeof(int32_t)));
  if (!ls->cap) LG_TRY(hipStreamCreateWithFlags(&ls->cap, hipStreamNonBlocking));
  for (hipEvent_t& e : ls->poll)
    if (!e) LG_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (hipEvent_t& e : ls->tev)
    if (!e) LG_TRY(hipEventCreate(&e));
  hipStream_t cap = ls->cap;
  double* db = ls->dbls.as<double>();

  LgArgs a{};
  a.n = n; a.m = m; a.meq = meq; a.wr = wr; a.wc = wc; a.nlr = nlr; a.nlc = nlc; a.nbr = nbr; a.nbc = nbc;
  a.ki = ib + o_ki; a.kpos = ib + o_kpos; a.kv = db + o_kv;
  a.ti = ib + o_ti; a.tpos = ib + o_tpos; a.tv = db + o_tv;
  a.lr = ib + o_lr; a.lrp = ib + o_lrp; a.lri = ib + o_lri; a.lrpos = ib + o_lrpos; a.lrv = db + o_lrv;
  a.lc = ib + o_lc; a.lcp = ib + o_lcp; a.lci = ib + o_lci; a.lcpos = ib + o_lcpos; a.lcv = db + o_lcv;
  a.rlong = fl; a.clong = fl + m;
  a.Tp = ib + o_Tp; a.Ti = ib + o_Ti; a.Tpos = ib + o_Tpos;
  a.Kp = b.indptr + orow; a.Kc = b.indices + onz; a.Kv = b.data + onz;
  a.c = b.c + on; a.q = b.q + om; a.l = b.l + on; a.u = b.u + on;
  a.dr = db + o_dr; a.dc = db + o_dc; a.cs = db + o_cs; a.ls = db + o_ls; a.us = db + o_us; a.qs = db + o_qs;
  a.tmpr = db + o_tmpr; a.tmpc = db + o_tmpc;
  a.x = db + o_x; a.xa = db + o_xa; a.xo = db + o_xo; a.xb = db + o_xb;
  a.y = db + o_y; a.ya = db + o_ya; a.yo = db + o_yo;
  a.part = db + o_part;
  a.hinv = hinv;
  a.st = ls->st.as<LgState>();
  a.eps = o.eps; a.eps_obj = o.eps_obj; a.rho = o.rho; a.b_suff = o.b_suff; a.b_nec = o.b_nec; a.b_art = o.b_art; a.theta = o.theta;
  a.step_safety = o.step_safety;
  a.chk = std::max(1, std::min(o.check_every, o.max_iters));
  a.kkt_every = std::max(1, o.kkt_every);
  a.max_iters = o.max_iters;
  a.warm = o.warm ? 1 : 0;
  a.ox = b.x + on; a.oy = b.y + om; a.ostats = b.stats + 4 * (int64_t)k; a.oist = b.istats + 2 * (int64_t)k;
  {
    double c0 = 0.0;
    LG_TRY(hipMemcpyAsync(&c0, b.c0 + k, sizeof(double), hipMemcpyDeviceToHost, s));
    LG_TRY(hipStreamSynchronize(s));
    a.c0 = c0;
  }

  hipEvent_t e0 = ls->tev[0], e1 = ls->tev[1], e2 = ls->tev[2];
  LG_TRY(hipEventRecord(e0, s));
  // ---- setup: scaling, scaled data, norms, power iteration, start point
  lg_ones<<<nbe, LB, 0, s>>>(a);
  for (int pass = 0; pass < o.ruiz_iters; ++pass) {
    lg_scale_pass<true><<<nbe, LB, 0, s>>>(a);
    lg_scale_apply<<<nbe, LB, 0, s>>>(a);
  }
  lg_scale_pass<false><<<nbe, LB, 0, s>>>(a);
  lg_scale_apply<<<nbe, LB, 0, s>>>(a);
  lg_fill<<<nbe, LB, 0, s>>>(a);
  lg_setup_norms<<<1, 1024, 0, s>>>(a, nbe);
  {
    double* v = a.x;   // scratch before the start point is written
    double* wv = a.y;
    std::vector<double> v0(n, 1.0 / std::sqrt((double)n));
    LG_TRY(hipMemcpyAsync(v, v0.data(), sizeof(double) * n, hipMemcpyHostToDevice, s));
    for (int it = 0; it < o.power_iters; ++it) {
      lg_pow_rows<<<nbr + nlr, LB, 0, s>>>(a, v, wv);
      lg_pow_cols<<<nbc + nlc, LB, 0, s>>>(a, wv, v);
      lg_pow_norm<<<1, 1024, 0, s>>>(a, nbc + nlc);
    }
    LG_TRY(hipStreamSynchronize(s));  // v0 is a host temporary
  }
  lg_start<<<nbe, LB, 0, s>>>(a);
  LG_TRY(hipGetLastError());
  LG_TRY(hipEventRecord(e1, s));

  // ---- one check period as a graph: chk iterations (the last one is the check iteration) + check
  GraphGuard gg;
  LG_TRY(hipStreamBeginCapture(cap, hipStreamCaptureModeRelaxed));
  for (int i = 0; i < a.chk; ++i) {
    if (i + 1 < a.chk) {
      lg_primal<false><<<nbc + nlc, LB, 0, cap>>>(a, i);
      lg_dual<false><<<nbr + nlr, LB, 0, cap>>>(a, i);
    } else {
      lg_primal<true><<<nbc + nlc, LB, 0, cap>>>(a, i);
      lg_dual<true><<<nbr + nlr, LB, 0, cap>>>(a, i);
    }
  }
  lg_kkt_rows<<<nbr + nlr, LB, 0, cap>>>(a);
  lg_kkt_cols<<<nbc + nlc, LB, 0, cap>>>(a);
  lg_check<<<1, 1024, 0, cap>>>(a);
  lg_restart<<<nbe, LB, 0, cap>>>(a);
  hipError_t ce = hipStreamEndCapture(cap, &gg.graph);
  if (ce != hipSuccess) {
    if (err) *err = std::string("graph capture: ") + hipGetErrorString(ce);
    return ce;
  }
  LG_TRY(hipGraphInstantiate(&gg.exec, gg.graph, nullptr, nullptr, 0));
  hipGraphExec_t exec = gg.exec;
  // replays: every kPoll replays the status is copied to pinned memory behind an event; the host waits on
  // the PREVIOUS poll's event, so kPoll..2*kPoll replays stay queued and the GPU never idles on the host
  constexpr int kPoll = 4;
  const int periods = (o.max_iters + a.chk - 1) / a.chk;
  hipError_t ge = hipSuccess;
  int32_t* ps = ls->pinned_status;
  ps[0] = ps[1] = -1;
  int pending = -1;  // slot of the outstanding poll
  for (int r = 0; r < periods && ge == hipSuccess; ++r) {
    ge = hipGraphLaunch(exec, s);
    if (ge != hipSuccess || (r + 1) % kPoll != 0) continue;
    const int slot = (r / kPoll) & 1;
    ge = hipMemcpyAsync(ps + slot, &a.st->status, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (ge == hipSuccess) ge = hipEventRecord(ls->poll[slot], s);
    if (ge != hipSuccess) break;
    if (pending >= 0) {
      ge = hipEventSynchronize(ls->poll[pending]);
      if (ge == hipSuccess && ps[pending] >= 0) break;
    }
    pending = slot;
  }
  if (ge == hipSuccess) lg_finish<<<nbe, LB, 0, s>>>(a);
  if (ge == hipSuccess) ge = hipGetLastError();
  if (ge == hipSuccess) ge = hipEventRecord(e2, s);
  if (ge == hipSuccess) ge = hipStreamSynchronize(s);
  if (ge != hipSuccess) {
    if (err) *err = std::string("large-LP PDHG: ") + hipGetErrorString(ge);
    return ge;
  }
  float t1 = 0, t2 = 0;
  (void)hipEventElapsedTime(&t1, e0, e1);
  (void)hipEventElapsedTime(&t2, e1, e2);
  if (setup_ms) *setup_ms += t1;
  if (pdhg_ms) *pdhg_ms += t2;
  return hipSuccess;
}

}  // namespace dvh

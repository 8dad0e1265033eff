// dvh_band.hip -- PDHG kernel for the battery-banded window LP (gfx950), the DER-VET hot path's common shape.
//
// Same algorithm, scaling and check logic as pdhg_ell_kernel (dvh_kernels.hip; restated in oracle/pdlp_ref.py),
// for windows whose CSR is the storagevet battery + DCM window (dervet/MicrogridScenario.py:319 solves it per
// window; SURVEY.md Appendix A, dervet_hip/lp/builder.py):
//   x = [ch(T), dis(T), ene(T), tau(J)],  J <= 4 demand periods in the window
//   row 0          ene_0                                      (= target)
//   row t+1        ch_t, dis_t, ene_t, ene_{t+1}               t = 0 .. T-2  (SOE recurrence)
//   row T          ch_{T-1}, dis_{T-1}, ene_{T-1}              (end-of-window target)
//   >= rows        ch_t, dis_t, tau_j                          at most one per step t (DCM epigraph)
//   bounds         ch, dis >= 0 (scaled lower bound exactly 0), objective coefficient of ene = 0
// The structure is detected and verified on the device from the CSR pattern (any values, any entry order
// within a row, DCM rows in any order); a window that does not match comes back with status kNeedsEll and
// is solved by the ELL kernel.
//
// Mapping: lane g owns S consecutive time steps t = S g + s -- their columns ch, dis, ene, their SOE rows and
// their DCM rows -- with every coefficient, bound, iterate and anchor in VGPRs.  An SpMV needs only the
// neighbour lane's first ene (K x) and last SOE-row dual (K^T y): one LDS store + one LDS load per lane and
// half-step instead of per-entry gathers.  The dense tau columns are summed by wave 0 from per-lane partials
// (no per-wave reduction).  With S = 2, 384 threads cover a 768-step monthly window in <= 168 VGPRs: two
// windows per CU, so one window's barrier and latency stalls are covered by the other window's work.
#include <type_traits>

#include "dvh_device.h"

namespace dvh {
namespace {

#ifndef DVH_BAND_S
#define DVH_BAND_S 1
#endif
constexpr int kBandS = DVH_BAND_S;    // steps per lane
constexpr int kBandB = 768 / kBandS;  // threads per window (T <= 768)
constexpr int kJMax = 4;      // tau (demand-period) columns per window
constexpr int kNeedsEll = -2;

// LDS layout in doubles (then ints): XE[B+1] YS[B+1] XT[kJMax] red[kNRed(NW+1)+4]
// TP[kJMax][B] XP[3S][B] YP[2S][B] | ints: dcm[S B] flag[4]
__host__ __device__ inline size_t band_lds_doubles(int B, int S) {
  const int NW = B / kWave;
  return 2 * (size_t)(B + 1) + kJMax + (size_t)kNRed * (NW + 1) + 4 + (size_t)kJMax * B +
         5 * (size_t)S * B;
}
__host__ __device__ inline size_t band_lds_bytes(int B, int S) {
  return align16(sizeof(double) * band_lds_doubles(B, S)) + align16(sizeof(int32_t) * ((size_t)S * B + 4));
}

// KKT pieces of one column / one row (out of line: the KKT check runs every 128 iterations, and inlined it
// would raise the whole kernel's register allocation)
struct ColKkt {
  double rd2, cx, bt;
};
__device__ __noinline__ ColKkt col_kkt_fn(double kt, double cj, double loj, double hij, double xj, double d) {
  const double rc = (cj - kt) / d;
  const bool fl = isfinite(loj), fh = isfinite(hij);
  const double lam = (fl && fh) ? rc : (fl ? fmax(rc, 0.0) : (fh ? fmin(rc, 0.0) : 0.0));
  const double rd = rc - lam;
  return {rd * rd, cj * xj, (fl ? loj * d * fmax(lam, 0.0) : 0.0) + (fh ? hij * d * fmin(lam, 0.0) : 0.0)};
}
__device__ __noinline__ double row_kkt_fn(double kv, double qi, double dr, int ge) {
  double r = (qi - kv) / dr;
  if (ge) r = fmax(r, 0.0);
  return r * r;
}

template <int B, int S>
__global__ __launch_bounds__(B, 3) void pdhg_band_kernel(const Batch b, const Work w, const Chunk ch, const Opts o) {
  constexpr int NW = B / kWave;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int k = ch.first + blockIdx.x;
  const int kl = blockIdx.x;
  const WinOff W = win_offsets(b, ch, k);
  const int n = W.n, m = W.m, meq = W.meq;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const double* scal = w.scal + (int64_t)kl * kScal;
  const int T = meq - 1, J = n - 3 * T, MI = m - meq;
  auto bail = [&]() {
    if (tid == 0) {
      b.istats[2 * k] = kNeedsEll;
      b.istats[2 * k + 1] = 0;
    }
  };
  if (scal[6] != 0.0 || T < 1 || T > S * B || J < 0 || J > kJMax || MI > T || (J == 0 && MI > 0)) {
    bail();
    return;
  }
  // ---- LDS carve
  double* XE = reinterpret_cast<double*>(smem);  // x-bar (x+) of ene at the lane's first step: [g]; [B] = 0
  double* YS = XE + (B + 1);                     // y (y+) of row S g: the init row (g = 0) / lane g-1's last SOE row
  double* XT = YS + (B + 1);                     // x-bar (x+) of the tau columns
  double* red = XT + kJMax;
  double* TP = red + kNRed * (NW + 1) + 4;       // [kJMax][B] per-lane partial K'y of the tau columns
  double* XP = TP + kJMax * B;                   // [3S][B] T(z) of the lane's columns (check iterations)
  double* YP = XP + 3 * S * B;                   // [2S][B] T(z) of the lane's rows
  int32_t* dcm = reinterpret_cast<int32_t*>(smem + align16(sizeof(double) * band_lds_doubles(B, S)));  // [S B]
  int32_t* flag = dcm + S * B;

  const int32_t* gkp = b.indptr + W.row;
  const int32_t* gkc = b.indices + W.nz;
  const double* gkv = w.kval + W.wz;
  const double* cs = w.cs + W.wn;
  const double* ls = w.ls + W.wn;
  const double* us = w.us + W.wn;
  const double* qs = w.qs + W.wm;
  const double* dcv = w.dc + W.wn;
  const double* drv = w.dr + W.wm;
  double* xo_g = b.x + W.on;
  double* yo_g = b.y + W.om;

  // ---- structure check (every entry of every row accounted for) and the step -> DCM row map
  for (int t = tid; t < S * B; t += B) dcm[t] = -1;
  if (tid == 0) flag[0] = 0;
  __syncthreads();
  int bad = 0;
  for (int r = tid; r <= T; r += B) {
    const int p0 = gkp[r], len = gkp[r + 1] - p0;
    if (r == 0) {
      bad |= !(len == 1 && gkc[p0] == 2 * T);
      continue;
    }
    const int t = r - 1;
    if (len != (r < T ? 4 : 3)) {
      bad = 1;
      continue;
    }
    unsigned seen = 0;
    for (int e = 0; e < len; ++e) {
      const int c = gkc[p0 + e];
      const int kind = c == t ? 0 : c == T + t ? 1 : c == 2 * T + t ? 2 : (r < T && c == 2 * T + t + 1) ? 3 : 4;
      if (kind == 4 || ((seen >> kind) & 1u)) bad = 1;
      seen |= 1u << kind;
    }
    // the kernel keeps no lower bound for ch / dis and no objective for ene
    bad |= ls[t] != 0.0 || ls[T + t] != 0.0 || cs[2 * T + t] != 0.0;
  }
  for (int i = meq + tid; i < m; i += B) {
    const int p0 = gkp[i], len = gkp[i + 1] - p0;
    if (len != 3) {
      bad = 1;
      continue;
    }
    int tc = -1, td = -1, jj = -1;
    for (int e = 0; e < 3; ++e) {
      const int c = gkc[p0 + e];
      if (c < T) {
        bad |= tc >= 0;
        tc = c;
      } else if (c < 2 * T) {
        bad |= td >= 0;
        td = c - T;
      } else if (c >= 3 * T && c < 3 * T + J) {
        bad |= jj >= 0;
        jj = c - 3 * T;
      } else {
        bad = 1;
      }
    }
    if (tc < 0 || td != tc || jj < 0) {
      bad = 1;
      continue;
    }
    if (atomicCAS(&dcm[tc], -1, i * 8 + jj) != -1) bad = 1;  // at most one DCM row per step
  }
  if (bad) flag[0] = 1;
  __syncthreads();
  if (flag[0] != 0) {
    bail();
    return;
  }

  // ---- the lane's steps t = S tid + s: columns ch, dis, ene (v = 0, 1, 2), SOE row t+1, DCM row -- in VGPRs
  double x[S][3], xa[S][3], hi[S][3];
  double cch[S], cdi[S], loe[S];  // objective of ch / dis, lower bound of ene
  double ks[S][4];                // SOE row: coefficients of ch_t, dis_t, ene_t, ene_{t+1}
  double kd[S][3];                // DCM row: coefficients of ch_t, dis_t, tau_j
  double ys[S], yas[S], qsr[S], yd[S], yad[S], qd[S];
  int drow[S], xta[S];            // DCM row index (-1: none), LDS address of XT[its tau]
  int jt[S];
  bool val[S];
  double kp = 0.0;                // coefficient of ene_{S tid} in row S tid (init row or lane tid-1's last SOE row)
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int t = S * tid + s;
    val[s] = t < T;
    drow[s] = -1;
    jt[s] = 0;
    cch[s] = cdi[s] = loe[s] = 0.0;
    ys[s] = yas[s] = qsr[s] = yd[s] = yad[s] = qd[s] = 0.0;
#pragma unroll
    for (int v = 0; v < 3; ++v) x[s][v] = xa[s][v] = hi[s][v] = kd[s][v] = 0.0;
#pragma unroll
    for (int v = 0; v < 4; ++v) ks[s][v] = 0.0;
    if (val[s]) {
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        hi[s][v] = us[v * T + t];
        x[s][v] = xa[s][v] = fmin(fmax(0.0, ls[v * T + t]), hi[s][v]);
      }
      cch[s] = cs[t];
      cdi[s] = cs[T + t];
      loe[s] = ls[2 * T + t];
      for (int p = gkp[t + 1]; p < gkp[t + 2]; ++p) {
        const int c = gkc[p];
        const double a = gkv[p];
        if (c == t) ks[s][0] = a;
        else if (c == T + t) ks[s][1] = a;
        else if (c == 2 * T + t) ks[s][2] = a;
        else ks[s][3] = a;
      }
      if (s == 0)
        for (int p = gkp[t]; p < gkp[t + 1]; ++p)
          if (gkc[p] == 2 * T + t) kp = gkv[p];
      qsr[s] = qs[t + 1];
      if (o.warm) {  // warm start from the unscaled x / y in the output buffers
#pragma unroll
        for (int v = 0; v < 3; ++v) {
          const int j = v * T + t;
          x[s][v] = xa[s][v] = fmin(fmax(xo_g[j] / dcv[j], ls[j]), hi[s][v]);
        }
        ys[s] = yas[s] = yo_g[t + 1] / drv[t + 1];
      }
      const int dv = dcm[t];
      if (dv >= 0) {
        drow[s] = dv >> 3;
        jt[s] = dv & 7;
        for (int p = gkp[drow[s]]; p < gkp[drow[s] + 1]; ++p) {
          const int c = gkc[p];
          const double a = gkv[p];
          if (c < T) kd[s][0] = a;
          else if (c < 2 * T) kd[s][1] = a;
          else kd[s][2] = a;
        }
        qd[s] = qs[drow[s]];
        if (o.warm) yd[s] = yad[s] = fmax(yo_g[drow[s]] / drv[drow[s]], 0.0);
      }
    }
    xta[s] = lds_addr(XT + jt[s]);
  }
  // Special state in wave 0 (registers sp[], meaning by lane): lane j < J holds tau column j {x, xa, c, lo, hi, x+};
  // lane kInitLane holds the init row (row 0: ene_0 = target) {y, ya, y+, q, coefficient, -}.
  constexpr int kInitLane = kWave - 1;
  static_assert(kJMax < kInitLane, "tau lanes and the init-row lane are distinct");
  const bool tlane = wid == 0 && lane < J, ilane = wid == 0 && lane == kInitLane;
  double sp[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (tlane) {
    const double l0 = ls[3 * T + lane], h0 = us[3 * T + lane];
    sp[0] = sp[1] = sp[5] = fmin(fmax(0.0, l0), h0);
    sp[2] = cs[3 * T + lane];
    sp[3] = l0;
    sp[4] = h0;
  }
  if (ilane) {
    sp[3] = qs[0];
    sp[4] = gkv[gkp[0]];
  }
  if (o.warm) {
    if (tlane) sp[0] = sp[1] = sp[5] = fmin(fmax(xo_g[3 * T + lane] / dcv[3 * T + lane], sp[3]), sp[4]);
    if (ilane) sp[0] = sp[1] = sp[2] = yo_g[0] / drv[0];
  }
  if (tid < kJMax) XT[tid] = 0.0;
  if (tid == 0) XE[B] = YS[B] = 0.0;
  XE[tid] = YS[tid] = 0.0;
  for (int u = tid; u < kJMax * B; u += B) TP[u] = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int v = 0; v < 3; ++v) XP[(3 * s + v) * B + tid] = x[s][v];
    YP[(2 * s) * B + tid] = ys[s];
    YP[(2 * s + 1) * B + tid] = yd[s];
  }
  __syncthreads();

  // ---- SpMV pieces (fixed summation order)
  // K^T of the lane's columns from its rows' values (vs: SOE rows, vd: DCM rows) and vprev = value of row S tid
  auto ktr = [&](const double (&vs)[S], const double (&vd)[S], double vprev, double (&out)[S][3]) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      out[s][0] = fma(kd[s][0], vd[s], ks[s][0] * vs[s]);
      out[s][1] = fma(kd[s][1], vd[s], ks[s][1] * vs[s]);
      out[s][2] = fma(ks[s][2], vs[s], s == 0 ? kp * vprev : ks[s > 0 ? s - 1 : 0][3] * vs[s > 0 ? s - 1 : 0]);
    }
  };
  // K of the lane's rows, own-column part (kfin adds the next lane's ene and the tau terms)
  auto kown = [&](const double (&v)[S][3], double (&os)[S], double (&od)[S]) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      os[s] = fma(ks[s][2], v[s][2], fma(ks[s][1], v[s][1], ks[s][0] * v[s][0]));
      if (s + 1 < S) os[s] = fma(ks[s][3], v[s + 1 < S ? s + 1 : s][2], os[s]);
      od[s] = fma(kd[s][1], v[s][1], kd[s][0] * v[s][0]);
    }
  };
  auto kfin = [&](double (&os)[S], double (&od)[S], double vnext) {
    os[S - 1] = fma(ks[S - 1][3], vnext, os[S - 1]);
#pragma unroll
    for (int s = 0; s < S; ++s) od[s] = fma(kd[s][2], lds_ld(xta[s]), od[s]);
  };
  // per-lane partial K'y of the tau columns from the DCM rows' values
  auto tau_parts = [&](const double (&vd)[S]) {
    if (J == 1) {
      double a = kd[0][2] * vd[0];
#pragma unroll
      for (int s = 1; s < S; ++s) a = fma(kd[s][2], vd[s], a);
      TP[tid] = a;
    } else {
      for (int j = 0; j < J; ++j) {
        double a = 0.0;
#pragma unroll
        for (int s = 0; s < S; ++s) a = fma(jt[s] == j ? kd[s][2] : 0.0, vd[s], a);
        TP[j * B + tid] = a;
      }
    }
  };
  // wave 0: lane j < J gets the sum over all lanes of TP[j][.] (fixed order; uniform per column)
  auto tau_kt = [&]() {
    double res = 0.0;
    for (int j = 0; j < J; ++j) {
      double a = 0.0;
#pragma unroll
      for (int r = 0; r < NW; ++r) a += TP[j * B + r * kWave + lane];
      a = uniform(wave_sum_dpp(a));
      if (lane == j) res = a;
    }
    return res;
  };

  // ---- ||Kt||_2 by power iteration (as the ELL kernel: v <- Kt'(Kt v), sigma^2 = |v_P| / |v_{P-1}|)
  double eta = scal[0];
  if (o.power_iters > 0) {
    const int P = o.power_iters;
    const double v0 = 1.0 / sqrt((double)n);
    double vc[S][3];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int v = 0; v < 3; ++v) vc[s][v] = val[s] ? v0 : 0.0;
    double vtau = (wid == 0 && lane < J) ? v0 : 0.0;
    double nv[2] = {0.0, 0.0};
    double ws[S], wd[S];
#pragma unroll
    for (int s = 0; s < S; ++s) ws[s] = wd[s] = 0.0;
    for (int pi = 0; pi <= P; ++pi) {
      if (pi > 0) {
        ktr(ws, wd, YS[tid], vc);
        if (wid == 0) {
          const double kt = tau_kt();
          vtau = lane < J ? kt : 0.0;
        }
      }
      if (pi >= P - 1) {
        double a = vtau * vtau;
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int v = 0; v < 3; ++v) a = fma(vc[s][v], vc[s][v], a);
        nv[pi - (P - 1)] = a;
      }
      if (pi == P) break;
      XE[tid] = vc[0][2];
      if (wid == 0 && lane < J) XT[lane] = vtau;
      __syncthreads();
      kown(vc, ws, wd);
      kfin(ws, wd, XE[tid + 1]);
      YS[tid + 1] = ws[S - 1];
      if (ilane) YS[0] = sp[4] * XE[0];
      tau_parts(wd);
      __syncthreads();
    }
    block_sum<B, 2>(nv, red);
    if (nv[0] > 0.0 && nv[1] > 0.0) eta = o.step_safety / sqrt(sqrt(nv[1] / nv[0]));
    YS[tid] = 0.0;
    if (tid == 0) YS[B] = 0.0;
    for (int u = tid; u < kJMax * B; u += B) TP[u] = 0.0;
    __syncthreads();
  }
  if (o.warm) {  // y images of the starting point
    YS[tid + 1] = ys[S - 1];
    if (ilane) YS[0] = sp[0];
    if (J > 0) tau_parts(yd);
    __syncthreads();
  }
  eta = uniform(eta);
  double pw = uniform(scal[1]);
  const double cnorm = uniform(scal[2]), qnorm = uniform(scal[3]), c0 = uniform(b.c0[k]);
  int it = 0, kin = 0, status = kIterLimit;
  double r0 = -1.0, rprev = -1.0;
  double* fin = red + kNRed * NW;
  if (tid == 0)
    for (int u = 0; u < 4; ++u) fin[u] = NAN;
  const int chk = o.check_every > 0 ? o.check_every : 64;
  double tau = uniform(eta / pw), sigma = uniform(eta * pw);
  const int kkt_every = o.kkt_every > 0 ? o.kkt_every : 1;
  int ck = chk, kk_ = kkt_every;
  int kbase = 0;
  auto hload = [&](int k0_) {
    const int kq = k0_ + lane;
    return kq < kHalpernTab ? w.hinv[kq] : 1.0 / (kq + 2.0);
  };
  double hw = hload(0);

  // wave 0 with one tau column: the tau reduction is interleaved with its own column work (straight-line code,
  // the partial loads are issued first); J >= 2 takes the generic per-column loop
  const bool w0 = wid == 0 && J == 1;
  double mv0, mv1, mv2, mv3;
  auto tau_update = [&](double kt, double ca, double cb, auto chk_tag) __attribute__((always_inline)) {
    constexpr bool CHECK = decltype(chk_tag)::value;
    if (tlane) {
      const double xo = sp[0], xan = sp[1];
      const double p1 = vmin(vmax(fma(-tau, sp[2] - kt, xo), sp[3]), sp[4]);
      const double xbt = fma(2.0, p1, -xo);
      XT[lane] = xbt;
      sp[0] = fma(ca, xbt, cb * xan);
      if (CHECK) {
        const double d = xo - p1, da = p1 - xan;
        mv0 += d * d;
        mv1 += da * da;
        sp[5] = p1;
      }
    }
  };
  auto iterate = [&](auto chk_tag, auto w0_tag) __attribute__((always_inline)) {
    constexpr bool CHECK = decltype(chk_tag)::value;
    constexpr bool W0 = decltype(w0_tag)::value;
    if (kin - kbase >= kWave) {
      kbase = kin;
      hw = hload(kin);
    }
    const double cb = readlane_f64(hw, kin - kbase), ca = 1.0 - cb;
    mv0 = mv1 = mv2 = mv3 = 0.0;
    // ---------------- primal half-step (reflected Halpern, rho = 1)
    double kxs[S], kxd[S];  // own-column part of K x-bar for the dual half-step
    {
      double ta0 = 0.0, ta1 = 0.0;
      if constexpr (W0) {
#pragma unroll
        for (int r = 0; r < NW; r += 2) {
          ta0 += TP[r * kWave + lane];
          if (r + 1 < NW) ta1 += TP[(r + 1) * kWave + lane];
        }
      }
      double kty[S][3], xb[S][3];
      ktr(ys, yd, YS[tid], kty);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const double cv[3] = {cch[s], cdi[s], 0.0};
        const double lv[3] = {0.0, 0.0, loe[s]};
#pragma unroll
        for (int v = 0; v < 3; ++v) {  // branch-free: padding steps have c = lo = hi = 0 and stay at 0
          const double p1 = vmin(vmax(fma(-tau, cv[v] - kty[s][v], x[s][v]), lv[v]), hi[s][v]);
          xb[s][v] = fma(2.0, p1, -x[s][v]);
          if (CHECK) {
            const double d = x[s][v] - p1, da = p1 - xa[s][v];
            mv0 += d * d;
            mv1 += da * da;
            XP[(3 * s + v) * B + tid] = p1;
          }
          x[s][v] = fma(ca, xb[s][v], cb * xa[s][v]);
        }
      }
      XE[tid] = xb[0][2];
      kown(xb, kxs, kxd);
      if constexpr (W0) {
        tau_update(uniform(wave_sum_dpp(ta0 + ta1)), ca, cb, chk_tag);
      } else {
        if (wid == 0 && J > 1) tau_update(tau_kt(), ca, cb, chk_tag);
      }
    }
    lds_barrier();
    // ---------------- dual half-step
    {
      kfin(kxs, kxd, XE[tid + 1]);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const double p1 = fma(sigma, qsr[s] - kxs[s], ys[s]);             // SOE row: equality
        const double p2 = vmax(fma(sigma, qd[s] - kxd[s], yd[s]), 0.0);  // DCM row: >=, its dual stays >= 0
        if (CHECK) {
          const double d = ys[s] - p1, da = p1 - yas[s], e = yd[s] - p2, ea = p2 - yad[s];
          mv2 += d * d + e * e;
          mv3 += da * da + ea * ea;
          YP[(2 * s) * B + tid] = p1;
          YP[(2 * s + 1) * B + tid] = p2;
        }
        ys[s] = fma(ca, fma(2.0, p1, -ys[s]), cb * yas[s]);
        yd[s] = fma(ca, fma(2.0, p2, -yd[s]), cb * yad[s]);
      }
      YS[tid + 1] = ys[S - 1];
      if (J > 0) tau_parts(yd);
      if (W0 || wid == 0) {  // init row (lane kInitLane): ene_0 = target
        if (ilane) {
          const double y0 = sp[0], ya0 = sp[1];
          const double q1 = fma(sigma, sp[3] - sp[4] * XE[0], y0);
          if (CHECK) {
            const double d = y0 - q1, da = q1 - ya0;
            mv2 += d * d;
            mv3 += da * da;
            sp[2] = q1;
          }
          const double yn = fma(ca, fma(2.0, q1, -y0), cb * ya0);
          sp[0] = yn;
          YS[0] = yn;
        }
      }
    }
    ++it;
    ++kin;
    lds_barrier();
  };

  using F = std::integral_constant<bool, false>;
  using Tt = std::integral_constant<bool, true>;
  while (it < o.max_iters) {
    if (--ck != 0) {
      if (w0)
        iterate(F(), Tt());
      else
        iterate(F(), F());
      continue;
    }
    ck = chk;
    if (w0)
      iterate(Tt(), Tt());
    else
      iterate(Tt(), F());
    // ---------------- check: fixed-point residual of z_k, restart test; every kkt_every-th check the relative
    // KKT error of T(z_k) in the unscaled space (as pdhg_ell_kernel)
    const bool kkt = (--kk_ == 0) || (it + chk > o.max_iters);
    if (kkt) kk_ = kkt_every;
    double acc[kNRed];
    acc[0] = mv0;
    acc[1] = mv1;
    acc[2] = mv2;
    acc[3] = mv3;
#pragma unroll
    for (int u = 4; u < kNRed; ++u) acc[u] = 0.0;
    if (kkt) {
      // images of T(z_k) in XE / XT / YS / TP (rewritten from z after the check)
      double xp[S][3], yps[S], ypd[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int v = 0; v < 3; ++v) xp[s][v] = XP[(3 * s + v) * B + tid];
        yps[s] = YP[(2 * s) * B + tid];
        ypd[s] = YP[(2 * s + 1) * B + tid];
      }
      XE[tid] = xp[0][2];
      YS[tid + 1] = yps[S - 1];
      if (ilane) YS[0] = sp[2];
      if (tlane) XT[lane] = sp[5];
      if (J > 0) tau_parts(ypd);
      lds_barrier();
      auto col_kkt = [&](int j, double kt, double cj, double loj, double hij, double xj) {
        const ColKkt r = col_kkt_fn(kt, cj, loj, hij, xj, dcv[opaque(j)]);
        acc[5] += r.rd2;
        acc[6] += r.cx;
        acc[8] += r.bt;
      };
      auto row_kkt = [&](int i, double kv, double qi, double yi, bool ge) {
        acc[4] += row_kkt_fn(kv, qi, drv[opaque(i)], ge);
        acc[7] += qi * yi;
      };
      double kt[S][3];
      ktr(yps, ypd, YS[tid], kt);
#pragma unroll
      for (int s = 0; s < S; ++s)
        if (val[s]) {
          const int t = S * tid + s;
          col_kkt(t, kt[s][0], cch[s], 0.0, hi[s][0], xp[s][0]);
          col_kkt(T + t, kt[s][1], cdi[s], 0.0, hi[s][1], xp[s][1]);
          col_kkt(2 * T + t, kt[s][2], 0.0, loe[s], hi[s][2], xp[s][2]);
        }
      if (wid == 0 && J > 0) {
        const double ktt = tau_kt();
        if (tlane) col_kkt(3 * T + lane, ktt, sp[2], sp[3], sp[4], sp[5]);
      }
      double kxs[S], kxd[S];
      kown(xp, kxs, kxd);
      kfin(kxs, kxd, XE[tid + 1]);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (val[s]) row_kkt(S * tid + s + 1, kxs[s], qsr[s], yps[s], false);
        if (drow[s] >= 0) row_kkt(drow[s], kxd[s], qd[s], ypd[s], true);
      }
      if (ilane) row_kkt(0, sp[4] * XE[0], sp[3], sp[2], false);
    }
    if (kkt) {
      block_sum1<B, kNRed, true>(acc, red);
    } else {
      double acc4[4] = {acc[0], acc[1], acc[2], acc[3]};
      block_sum1<B, 4, true>(acc4, red);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = acc4[u];
    }
    if (kkt) {
      const double pobj = acc[6] + c0, dobj = acc[7] + acc[8] + c0;
      const double pres = sqrt(acc[4]) / (1.0 + qnorm), dres = sqrt(acc[5]) / (1.0 + cnorm);
      const double gap = fabs(pobj - dobj) / (1.0 + fabs(pobj) + fabs(dobj));
      if (tid == 0) {
        fin[0] = pobj;
        fin[1] = pres;
        fin[2] = dres;
        fin[3] = gap;
      }
      if (pres <= o.eps && dres <= o.eps && gap <= o.eps) {
        status = kOptimal;
        break;
      }
      if (!(isfinite(pobj) && isfinite(dobj))) {
        status = kNumerical;
        break;
      }
    }
    const double r = sqrt(pw * acc[0] + acc[2] / pw);
    if (r0 < 0.0) r0 = r;
    const bool restart = (r <= o.b_suff * r0) || (r <= o.b_nec * r0 && rprev >= 0.0 && r > rprev) ||
                         ((double)kin >= o.b_art * (double)it);
    if (restart) {
      const double ddx = sqrt(acc[1]), ddy = sqrt(acc[3]);
      if (ddx > 1e-10 && ddy > 1e-10) pw = uniform(pw_update(ddy / ddx, pw, o.theta));
      tau = uniform(eta / pw);
      sigma = uniform(eta * pw);
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int v = 0; v < 3; ++v) x[s][v] = xa[s][v] = XP[(3 * s + v) * B + tid];
        ys[s] = yas[s] = YP[(2 * s) * B + tid];
        yd[s] = yad[s] = YP[(2 * s + 1) * B + tid];
      }
      if (ilane) sp[0] = sp[1] = sp[2];
      if (tlane) sp[0] = sp[1] = sp[5];
      kin = 0;
      kbase = 0;
      hw = hload(0);
      r0 = r;
      rprev = -1.0;
    } else {
      rprev = r;
    }
    if (restart || kkt) {  // the y images must hold z again (after a restart z = T(z_k))
      YS[tid + 1] = ys[S - 1];
      if (ilane) YS[0] = sp[0];
      if (J > 0) tau_parts(yd);
    }
    lds_barrier();
  }
  // outputs: the last check's T(z_k), unscaled
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (val[s]) {
      const int t = S * tid + s;
#pragma unroll
      for (int v = 0; v < 3; ++v) xo_g[v * T + t] = XP[(3 * s + v) * B + tid] * dcv[v * T + t];
      yo_g[t + 1] = YP[(2 * s) * B + tid] * drv[t + 1];
      if (drow[s] >= 0) yo_g[drow[s]] = YP[(2 * s + 1) * B + tid] * drv[drow[s]];
    }
  if (tlane) xo_g[3 * T + lane] = sp[5] * dcv[3 * T + lane];
  if (ilane) yo_g[0] = sp[2] * drv[0];
  if (tid == 0) {
    b.istats[2 * k] = status;
    b.istats[2 * k + 1] = it;
    for (int u = 0; u < 4; ++u) b.stats[4 * k + u] = fin[u];
  }
}

}  // namespace

hipError_t launch_pdhg_band(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s) {
  constexpr int B = kBandB, S = kBandS;
  const size_t lds = band_lds_bytes(B, S);
  auto kern = pdhg_band_kernel<B, S>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(ch.count), dim3(B), lds, s, b, w, ch, o);
  return hipGetLastError();
}

}  // namespace dvh

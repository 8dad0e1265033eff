// dvh_band.hip -- PDHG kernel for the battery-banded window LP (gfx950), the DER-VET hot path's common shape.
//
// Same algorithm, scaling and check logic as pdhg_ell_kernel (dvh_kernels.hip; restated in oracle/pdlp_ref.py),
// for windows whose CSR is the storagevet battery + DCM window (dervet/MicrogridScenario.py:319 solves it per
// window; SURVEY.md Appendix A, dervet_hip/lp/builder.py), optionally with an LP-relaxed ICE (ICE = true):
//   x = [ch(T), dis(T), ene(T), tau(J)] (+ [elec(T), on(T)]),  J <= 4 demand periods in the window
//   row 0          ene_0                                      (= target)
//   row t+1        ch_t, dis_t, ene_t, ene_{t+1}               t = 0 .. T-2  (SOE recurrence)
//   row T          ch_{T-1}, dis_{T-1}, ene_{T-1}              (end-of-window target)
//   >= rows        ch_t, dis_t, tau_j (+ elec_t)               at most one per step t (DCM epigraph)
//   >= rows (ICE)  elec_t, on_t                                exactly two per step (rated / minimum power,
//                                                              RotatingGeneratorSizing.py:110-136)
//   bounds         ch, dis (, elec, on) >= 0 (scaled lower bound exactly 0)
// The structure is detected and verified on the device from the CSR pattern (any values, any entry order
// within a row, >= rows in any order); a window that does not match comes back with status kNeedsEll.
//
// Mapping: lane t owns time step t -- its columns, its SOE / DCM (/ ICE) rows -- with every coefficient, bound,
// objective, iterate and anchor in VGPRs.  An SpMV needs only the next step's ene (K x) and the previous SOE
// row's dual (K^T y): one LDS store + one LDS load per lane and half-step instead of per-entry gathers.  The
// dense tau columns are summed by wave 0 from per-lane partials (no per-wave reduction).  768 threads per
// window, 12 waves, <= 168 VGPRs.
#include <type_traits>

#include "dvh_device.h"

namespace dvh {
namespace {

constexpr int kBandB = 768;   // threads per window (T <= kBandB steps)
constexpr int kJMax = 4;      // tau (demand-period) columns per window
constexpr int kNeedsEll = -2;

// LDS layout in doubles (then ints): XE[B+1] YS[B+1] XT[kJMax] red[kNRed(NW+1)+4] TP[kJMax][B] XP[NC][B] YP[NR][B]
// (ICE: RO[6][B]) | ints: dcm[B] ice_a[B] ice_b[B] ice_n[B] flag[4]
__host__ __device__ inline size_t band_lds_doubles(int B, bool ice) {
  const int NW = B / kWave, NC = ice ? 5 : 3, NR = ice ? 4 : 2;
  return 2 * (size_t)(B + 1) + kJMax + (size_t)kNRed * (NW + 1) + 4 + (size_t)kJMax * B + (size_t)(NC + NR) * B +
         (ice ? 6 * (size_t)B : 0);
}
__host__ __device__ inline size_t band_lds_bytes(int B, bool ice) {
  return align16(sizeof(double) * band_lds_doubles(B, ice)) + align16(sizeof(int32_t) * (4 * (size_t)B + 4));
}

// KKT pieces of one column / one row (out of line: the KKT check runs every 128 iterations, and inlined it
// would raise the whole kernel's register allocation).  d / dr: the column / row scaling, id / idr: their
// reciprocals from the setup kernel (the unscaling is a multiplication, not a division)
struct ColKkt {
  double rd2, cx, bt;
};
__device__ __noinline__ ColKkt col_kkt_fn(double kt, double cj, double loj, double hij, double xj, double d,
                                          double id) {
  const double rc = (cj - kt) * id;
  const bool fl = isfinite(loj), fh = isfinite(hij);
  const double lam = (fl && fh) ? rc : (fl ? fmax(rc, 0.0) : (fh ? fmin(rc, 0.0) : 0.0));
  const double rd = rc - lam;
  return {rd * rd, cj * xj, (fl ? loj * d * fmax(lam, 0.0) : 0.0) + (fh ? hij * d * fmin(lam, 0.0) : 0.0)};
}
struct RowKkt {
  double rp2, y2;
};
__device__ __noinline__ RowKkt row_kkt_fn(double kv, double qi, double yi, double dr, double idr, int ge) {
  double r = (qi - kv) * idr;
  if (ge) r = fmax(r, 0.0);
  return {r * r, (yi * dr) * (yi * dr)};
}

template <int B, bool ICE>
__global__ __launch_bounds__(B, 3) void pdhg_band_kernel(const Batch b, const Work w, const Chunk ch, const Opts o,
                                                        const int32_t* list) {
  constexpr int NW = B / kWave;
  constexpr int NC = ICE ? 5 : 3;  // columns per step: ch, dis, ene (, elec, on)
  constexpr int NR = ICE ? 4 : 2;  // rows per step: SOE, DCM (, ICE rated, ICE minimum)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int k = list ? list[blockIdx.x] : ch.first + (int)blockIdx.x;
  const int kl = k - ch.first;
  const WinOff W = win_offsets(b, ch, k);
  const int n = W.n, m = W.m, meq = W.meq;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const double* scal = w.scal + (int64_t)kl * kScal;
  const int T = meq - 1, J = n - (ICE ? 5 : 3) * T, MI = m - meq;
  const int MD = ICE ? MI - 2 * T : MI;  // DCM rows
  auto bail = [&]() {
    if (tid == 0) {
      b.istats[2 * k] = kNeedsEll;
      b.istats[2 * k + 1] = 0;
    }
  };
  if (scal[6] == 3.0) return;  // reported infeasible by the setup kernel
  if (scal[6] != 0.0 || T < 1 || T > B || J < 0 || J > kJMax || MD < 0 || MD > T || (J == 0 && MD > 0)) {
    bail();
    return;
  }
  const int CE = 3 * T + J, CO = 4 * T + J;  // first elec / on column (ICE)
  // ---- LDS carve
  double* XE = reinterpret_cast<double*>(smem);  // x-bar (x+) of ene_t at [t]; [T..B] stay 0
  double* YS = XE + (B + 1);                     // y (y+) of row t at [t]: the init row (t = 0), SOE row of step t-1
  double* XT = YS + (B + 1);                     // x-bar (x+) of the tau columns
  double* red = XT + kJMax;
  double* TP = red + kNRed * (NW + 1) + 4;       // [kJMax][B] per-lane partial K'y of the tau columns
  double* XP = TP + kJMax * B;                   // [NC][B] T(z) of the lane's columns (check iterations)
  double* YP = XP + NC * B;                      // [NR][B] T(z) of the lane's rows
  // ICE: read-only data of the ICE columns / rows in LDS instead of VGPRs (the register budget at 3 waves per
  // SIMD is 168): RO[0..1][.] = c of elec / on, RO[2..3][.] = upper bound of elec / on, RO[4..5][.] = q of the
  // two ICE rows
  double* RO = YP + NR * B;
  int32_t* dcm = reinterpret_cast<int32_t*>(smem + align16(sizeof(double) * band_lds_doubles(B, ICE)));  // [B]
  int32_t* ice_a = dcm + B;   // [B] ICE rows of each step (lower / higher row index), and their count
  int32_t* ice_b = ice_a + B;
  int32_t* ice_n = ice_b + B;
  int32_t* flag = ice_n + B;

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

  // ---- structure check (every entry of every row accounted for) and the step -> row maps
  dcm[tid] = -1;
  ice_a[tid] = 0x7fffffff;
  ice_b[tid] = -1;
  ice_n[tid] = 0;
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
    // the kernel keeps no lower bound for ch / dis (/ elec / on)
    bad |= ls[t] != 0.0 || ls[T + t] != 0.0;
    if (ICE) bad |= ls[CE + t] != 0.0 || ls[CO + t] != 0.0;
  }
  for (int i = meq + tid; i < m; i += B) {
    const int p0 = gkp[i], len = gkp[i + 1] - p0;
    if (ICE && len == 2) {  // ICE row: elec_t, on_t
      int te = -1, to = -1;
      for (int e = 0; e < 2; ++e) {
        const int c = gkc[p0 + e];
        if (c >= CE && c < CE + T) te = c - CE;
        else if (c >= CO && c < CO + T) to = c - CO;
      }
      if (te < 0 || te != to) {
        bad = 1;
        continue;
      }
      atomicMin(&ice_a[te], i);
      atomicMax(&ice_b[te], i);
      atomicAdd(&ice_n[te], 1);
      continue;
    }
    if (len != (ICE ? 4 : 3)) {
      bad = 1;
      continue;
    }
    int tc = -1, td = -1, jj = -1, te = ICE ? -1 : -2;
    for (int e = 0; e < len; ++e) {
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
      } else if (ICE && c >= CE && c < CE + T) {
        bad |= te >= 0;
        te = c - CE;
      } else {
        bad = 1;
      }
    }
    if (tc < 0 || td != tc || jj < 0 || (ICE && te != tc)) {
      bad = 1;
      continue;
    }
    if (atomicCAS(&dcm[tc], -1, i * 8 + jj) != -1) bad = 1;  // at most one DCM row per step
  }
  if (bad) flag[0] = 1;
  __syncthreads();
  if (ICE && tid < T && ice_n[tid] != 2) flag[0] = 1;  // exactly two ICE rows per step
  __syncthreads();
  if (flag[0] != 0) {
    bail();
    return;
  }

  // ---- the lane's step t: columns (v) ch, dis, ene (, elec, on), rows (r) SOE, DCM (, ICE a, ICE b) -- VGPRs
  const int t = tid;
  const bool val = t < T;
  auto col = [&](int v) { return v < 3 ? v * T + t : (v == 3 ? CE : CO) + t; };
  double x[NC], xa[NC], cc[3], hi[3];
  double loe = 0.0;                        // lower bound of ene (the others are 0)
  double ks[4] = {0.0, 0.0, 0.0, 0.0};     // SOE row: coefficients of ch_t, dis_t, ene_t, ene_{t+1}
  double kd[4] = {0.0, 0.0, 0.0, 0.0};     // DCM row: coefficients of ch_t, dis_t, tau_j, elec_t
  double ka[2] = {0.0, 0.0}, kb[2] = {0.0, 0.0};  // ICE rows: coefficients of elec_t, on_t
  double kp = 0.0;                         // coefficient of ene_t in row t (init row or SOE row of step t-1)
  double y[NR], ya[NR], q[2];
  int drow = -1, jt = 0, ra = -1, rb = -1;
#pragma unroll
  for (int v = 0; v < NC; ++v) x[v] = xa[v] = 0.0;
#pragma unroll
  for (int v = 0; v < 3; ++v) cc[v] = hi[v] = 0.0;
#pragma unroll
  for (int r = 0; r < NR; ++r) y[r] = ya[r] = 0.0;
  q[0] = q[1] = 0.0;
  if (ICE)
    for (int u = 0; u < 6; ++u) RO[u * B + tid] = 0.0;
  auto cof = [&](int v) -> double { return v < 3 ? cc[v] : RO[(v - 3) * B + tid]; };
  auto hib = [&](int v) -> double { return v < 3 ? hi[v] : RO[(v - 1) * B + tid]; };
  auto rhs = [&](int r) -> double { return r < 2 ? q[r] : RO[(r + 2) * B + tid]; };
  if (val) {
#pragma unroll
    for (int v = 0; v < NC; ++v) {
      const int j = col(v);
      if (v < 3) {
        hi[v] = us[j];
        cc[v] = cs[j];
      } else {
        RO[(v - 1) * B + tid] = us[j];
        RO[(v - 3) * B + tid] = cs[j];
      }
      x[v] = xa[v] = fmin(fmax(0.0, ls[j]), us[j]);
    }
    loe = ls[2 * T + t];
    for (int p = gkp[t + 1]; p < gkp[t + 2]; ++p) {
      const int c = gkc[p];
      const double a = gkv[p];
      if (c == t) ks[0] = a;
      else if (c == T + t) ks[1] = a;
      else if (c == 2 * T + t) ks[2] = a;
      else ks[3] = a;
    }
    for (int p = gkp[t]; p < gkp[t + 1]; ++p)
      if (gkc[p] == 2 * T + t) kp = gkv[p];
    q[0] = qs[t + 1];
    const int dv = dcm[t];
    if (dv >= 0) {
      drow = dv >> 3;
      jt = dv & 7;
      for (int p = gkp[drow]; p < gkp[drow + 1]; ++p) {
        const int c = gkc[p];
        const double a = gkv[p];
        if (c < T) kd[0] = a;
        else if (c < 2 * T) kd[1] = a;
        else if (c < 3 * T + J) kd[2] = a;
        else kd[3] = a;
      }
      q[1] = qs[drow];
    }
    if (ICE) {
      ra = ice_a[t];
      rb = ice_b[t];
      for (int p = gkp[ra]; p < gkp[ra + 1]; ++p) (gkc[p] < CO ? ka[0] : ka[1]) = gkv[p];
      for (int p = gkp[rb]; p < gkp[rb + 1]; ++p) (gkc[p] < CO ? kb[0] : kb[1]) = gkv[p];
      RO[4 * B + tid] = qs[ra];
      RO[5 * B + tid] = qs[rb];
    }
    if (o.warm) {  // warm start from the unscaled x / y in the output buffers
#pragma unroll
      for (int v = 0; v < NC; ++v) {
        const int j = col(v);
        x[v] = xa[v] = fmin(fmax(xo_g[j] / dcv[j], ls[j]), us[j]);
      }
      y[0] = ya[0] = yo_g[t + 1] / drv[t + 1];
      if (drow >= 0) y[1] = ya[1] = fmax(yo_g[drow] / drv[drow], 0.0);
      if (ICE) {
        y[2] = ya[2] = fmax(yo_g[ra] / drv[ra], 0.0);
        y[3] = ya[3] = fmax(yo_g[rb] / drv[rb], 0.0);
      }
    }
  }
  const int xta = lds_addr(XT + jt);
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
  for (int v = 0; v < NC; ++v) XP[v * B + tid] = x[v];
#pragma unroll
  for (int r = 0; r < NR; ++r) YP[r * B + tid] = y[r];
  __syncthreads();

  // ---- SpMV pieces (fixed summation order)
  // K^T of the lane's columns from its rows' values vr and vprev = the value of row t
  auto ktr = [&](const double (&vr)[NR], double vprev, double (&out)[NC]) {
    out[0] = fma(kd[0], vr[1], ks[0] * vr[0]);
    out[1] = fma(kd[1], vr[1], ks[1] * vr[0]);
    out[2] = fma(ks[2], vr[0], kp * vprev);
    if constexpr (ICE) {
      out[3] = fma(kb[0], vr[3], fma(ka[0], vr[2], kd[3] * vr[1]));
      out[4] = fma(kb[1], vr[3], ka[1] * vr[2]);
    }
  };
  // K of the lane's rows, own-column part (kfin adds the next step's ene and the tau term)
  auto kown = [&](const double (&v)[NC], double (&os)[NR]) {
    os[0] = fma(ks[2], v[2], fma(ks[1], v[1], ks[0] * v[0]));
    os[1] = fma(kd[1], v[1], kd[0] * v[0]);
    if constexpr (ICE) {
      os[1] = fma(kd[3], v[3], os[1]);
      os[2] = fma(ka[1], v[4], ka[0] * v[3]);
      os[3] = fma(kb[1], v[4], kb[0] * v[3]);
    }
  };
  auto kfin = [&](double (&os)[NR], double vnext) {
    os[0] = fma(ks[3], vnext, os[0]);
    os[1] = fma(kd[2], lds_ld(xta), os[1]);
  };
  // The iteration's forms with the objective / right-hand side folded into the FMA chains: K^T y - c for the
  // primal half-step (x + tau (K^T y - c) = x - tau (c - K^T y)) and K x - q for the dual one (y - sigma (K x - q)):
  // one FP64 operation fewer per column and per row than forming the difference afterwards.
  auto ktr_c = [&](const double (&vr)[NR], double vprev, double (&out)[NC]) {
    out[0] = fma(kd[0], vr[1], fma(ks[0], vr[0], -cof(0)));
    out[1] = fma(kd[1], vr[1], fma(ks[1], vr[0], -cof(1)));
    out[2] = fma(ks[2], vr[0], fma(kp, vprev, -cof(2)));
    if constexpr (ICE) {
      out[3] = fma(kb[0], vr[3], fma(ka[0], vr[2], fma(kd[3], vr[1], -cof(3))));
      out[4] = fma(kb[1], vr[3], fma(ka[1], vr[2], -cof(4)));
    }
  };
  auto kown_q = [&](const double (&v)[NC], double (&os)[NR]) {
    os[0] = fma(ks[2], v[2], fma(ks[1], v[1], fma(ks[0], v[0], -q[0])));
    os[1] = fma(kd[1], v[1], fma(kd[0], v[0], -q[1]));
    if constexpr (ICE) {
      os[1] = fma(kd[3], v[3], os[1]);
      os[2] = fma(ka[1], v[4], fma(ka[0], v[3], -rhs(2)));
      os[3] = fma(kb[1], v[4], fma(kb[0], v[3], -rhs(3)));
    }
  };
  // per-lane partial K'y of the tau columns from the DCM row's value
  auto tau_parts = [&](double vd) {
    if (J == 1) {
      TP[tid] = kd[2] * vd;
    } else {
      for (int j = 0; j < J; ++j) TP[j * B + tid] = (jt == j ? kd[2] : 0.0) * vd;
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
    double vc[NC];
#pragma unroll
    for (int v = 0; v < NC; ++v) vc[v] = val ? v0 : 0.0;
    double vtau = (wid == 0 && lane < J) ? v0 : 0.0;
    double nv[2] = {0.0, 0.0};
    double wr[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) wr[r] = 0.0;
    for (int pi = 0; pi <= P; ++pi) {
      if (pi > 0) {
        ktr(wr, YS[tid], vc);
        if (wid == 0) {
          const double kt = tau_kt();
          vtau = lane < J ? kt : 0.0;
        }
      }
      if (pi >= P - 1) {
        double a = vtau * vtau;
#pragma unroll
        for (int v = 0; v < NC; ++v) a = fma(vc[v], vc[v], a);
        nv[pi - (P - 1)] = a;
      }
      if (pi == P) break;
      XE[tid] = vc[2];
      if (wid == 0 && lane < J) XT[lane] = vtau;
      __syncthreads();
      kown(vc, wr);
      kfin(wr, XE[tid + 1]);
      YS[tid + 1] = wr[0];
      if (ilane) YS[0] = sp[4] * XE[0];
      tau_parts(wr[1]);
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
    YS[tid + 1] = y[0];
    if (ilane) YS[0] = sp[0];
    if (J > 0) tau_parts(y[1]);
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
    double kx[NR];  // own-column part of K x-bar for the dual half-step
    {
      double ta0 = 0.0, ta1 = 0.0;
      if constexpr (W0) {
#pragma unroll
        for (int r = 0; r < NW; r += 2) {
          ta0 += TP[r * kWave + lane];
          if (r + 1 < NW) ta1 += TP[(r + 1) * kWave + lane];
        }
      }
      double kty[NC], xb[NC];
      ktr_c(y, YS[tid], kty);
#pragma unroll
      for (int v = 0; v < NC; ++v) {  // branch-free: padding steps have c = lo = hi = 0 and stay at 0
        const double lo = v == 2 ? loe : 0.0;
        const double p1 = vmin(vmax(fma(tau, kty[v], x[v]), lo), hib(v));
        xb[v] = fma(2.0, p1, -x[v]);
        if (CHECK) {
          const double d = x[v] - p1, da = p1 - xa[v];
          mv0 += d * d;
          mv1 += da * da;
          XP[v * B + tid] = p1;
        }
        x[v] = fma(ca, xb[v], cb * xa[v]);
      }
      XE[tid] = xb[2];
      kown_q(xb, kx);
      if constexpr (W0) {
        tau_update(uniform(wave_sum_dpp(ta0 + ta1)), ca, cb, chk_tag);
      } else {
        if (wid == 0 && J > 1) tau_update(tau_kt(), ca, cb, chk_tag);
      }
    }
    lds_barrier();
    // ---------------- dual half-step
    {
      kfin(kx, XE[tid + 1]);
#pragma unroll
      for (int r = 0; r < NR; ++r) {  // row 0 (SOE) is an equality; DCM / ICE rows are >=: duals stay >= 0
        double p1 = fma(-sigma, kx[r], y[r]);
        if (r > 0) p1 = vmax(p1, 0.0);
        if (CHECK) {
          const double d = y[r] - p1, da = p1 - ya[r];
          mv2 += d * d;
          mv3 += da * da;
          YP[r * B + tid] = p1;
        }
        y[r] = fma(ca, fma(2.0, p1, -y[r]), cb * ya[r]);
      }
      YS[tid + 1] = y[0];
      if (J > 0) tau_parts(y[1]);
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
      double xp[NC], yp[NR];
#pragma unroll
      for (int v = 0; v < NC; ++v) xp[v] = XP[v * B + tid];
#pragma unroll
      for (int r = 0; r < NR; ++r) yp[r] = YP[r * B + tid];
      XE[tid] = xp[2];
      YS[tid + 1] = yp[0];
      if (ilane) YS[0] = sp[2];
      if (tlane) XT[lane] = sp[5];
      if (J > 0) tau_parts(yp[1]);
      lds_barrier();
      auto col_kkt = [&](int j, double kt, double cj, double loj, double hij, double xj) {
        const int jj = opaque(j);
        const ColKkt r = col_kkt_fn(kt, cj, loj, hij, xj, dcv[jj], w.tmpc[W.wn + jj]);
        acc[5] += r.rd2;
        acc[6] += r.cx;
        acc[8] += r.bt;
      };
      auto row_kkt = [&](int i, double kv, double qi, double yi, bool ge) {
        const int ii = opaque(i);
        const RowKkt r = row_kkt_fn(kv, qi, yi, drv[ii], w.tmpr[W.wm + ii], ge);
        acc[4] += r.rp2;
        acc[7] += qi * yi;
        acc[9] += r.y2;
      };
      double kt[NC];
      ktr(yp, YS[tid], kt);
      if (val) {
#pragma unroll
        for (int v = 0; v < NC; ++v) col_kkt(col(v), kt[v], cof(v), v == 2 ? loe : 0.0, hib(v), xp[v]);
      }
      if (wid == 0 && J > 0) {
        const double ktt = tau_kt();
        if (tlane) col_kkt(3 * T + lane, ktt, sp[2], sp[3], sp[4], sp[5]);
      }
      double kv[NR];
      kown(xp, kv);
      kfin(kv, XE[tid + 1]);
      if (val) row_kkt(t + 1, kv[0], q[0], yp[0], false);
      if (drow >= 0) row_kkt(drow, kv[1], q[1], yp[1], true);
      if (ICE && val) {
        row_kkt(ra, kv[2], rhs(2), yp[2], true);
        row_kkt(rb, kv[3], rhs(3), yp[3], true);
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
      if (kkt_done(o, pres, dres, gap, pobj, dobj, acc[4], acc[9])) {
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
      for (int v = 0; v < NC; ++v) x[v] = xa[v] = XP[v * B + tid];
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) y[rr] = ya[rr] = YP[rr * B + tid];
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
      YS[tid + 1] = y[0];
      if (ilane) YS[0] = sp[0];
      if (J > 0) tau_parts(y[1]);
    }
    lds_barrier();
  }
  // outputs: the last check's T(z_k), unscaled
  if (val) {
#pragma unroll
    for (int v = 0; v < NC; ++v) xo_g[col(v)] = XP[v * B + tid] * dcv[col(v)];
    yo_g[t + 1] = YP[tid] * drv[t + 1];
    if (drow >= 0) yo_g[drow] = YP[B + tid] * drv[drow];
    if (ICE) {
      yo_g[ra] = YP[2 * B + tid] * drv[ra];
      yo_g[rb] = YP[3 * B + tid] * drv[rb];
    }
  }
  if (tlane) xo_g[3 * T + lane] = sp[5] * dcv[3 * T + lane];
  if (ilane) yo_g[0] = sp[2] * drv[0];
  if (tid == 0) {
    b.istats[2 * k] = status;
    b.istats[2 * k + 1] = it;
    for (int u = 0; u < 4; ++u) b.stats[4 * k + u] = fin[u];
  }
}

template <bool ICE>
hipError_t launch_band_one(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s,
                           const int32_t* list, int nlist) {
  constexpr int B = kBandB;
  const size_t lds = band_lds_bytes(B, ICE);
  auto kern = pdhg_band_kernel<B, ICE>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(list ? nlist : ch.count), dim3(B), lds, s, b, w, ch, o, list);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_pdhg_band(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s, bool ice,
                            const int32_t* list, int nlist) {
  return ice ? launch_band_one<true>(b, w, ch, o, s, list, nlist) : launch_band_one<false>(b, w, ch, o, s, list, nlist);
}

}  // namespace dvh

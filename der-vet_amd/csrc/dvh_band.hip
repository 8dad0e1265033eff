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
// Mapping: lane t owns time step t -- its three columns, its SOE row and its DCM row -- with every coefficient,
// bound, iterate and anchor in VGPRs (<= 80: six waves per SIMD, i.e. two 768-thread windows per CU, so one
// window's barrier stalls are covered by the other's work).  An SpMV needs only the neighbour step's ene
// (K x) and SOE-row dual (K^T y): one LDS store + one LDS load per lane and half-step instead of per-entry
// gathers.  The dense tau columns are summed by wave 0 from per-lane partials (no per-wave reduction).
#include <type_traits>

#include "dvh_device.h"

namespace dvh {
namespace {

constexpr int kBandB = 768;   // threads per window (T <= kBandB steps)
constexpr int kJMax = 4;      // tau (demand-period) columns per window
constexpr int kNeedsEll = -2;

// LDS layout in doubles (then ints): XE[B+1] YS[B+1] XT[kJMax] TS[6][kJMax] I0[8] red[kNRed(NW+1)+4]
// TP[kJMax][B] XP[3][B] YP[2][B] | ints: dcm[B] flag[4]
__host__ __device__ inline size_t band_lds_doubles(int B) {
  const int NW = B / kWave;
  return 2 * (size_t)(B + 1) + 7 * kJMax + 8 + (size_t)kNRed * (NW + 1) + 4 + (size_t)kJMax * B + 5 * (size_t)B;
}
__host__ __device__ inline size_t band_lds_bytes(int B) {
  return align16(sizeof(double) * band_lds_doubles(B)) + align16(sizeof(int32_t) * ((size_t)B + 4));
}

template <int B>
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
  if (scal[6] != 0.0 || T < 1 || T > B || J < 0 || J > kJMax || MI > T || (J == 0 && MI > 0)) {
    bail();
    return;
  }
  // ---- LDS carve
  double* XE = reinterpret_cast<double*>(smem);  // x-bar (x+) of ene_t at [t]; [T..B] stay 0
  double* YS = XE + (B + 1);                     // y (y+) of row t at [t]: the init row (t = 0), SOE row of step t-1
  double* XT = YS + (B + 1);                     // x-bar (x+) of the tau columns
  double* TS = XT + kJMax;                       // tau state [6][kJMax]: x, xa, c, lo, hi, x+
  double* I0 = TS + 6 * kJMax;                   // init row: y, ya, y+, q, coefficient
  double* red = I0 + 8;
  double* TP = red + kNRed * (NW + 1) + 4;       // [kJMax][B] per-lane partial K'y of the tau columns
  double* XP = TP + kJMax * B;                   // [3][B] T(z) of the lane's columns (check iterations)
  double* YP = XP + 3 * B;                       // [2][B] T(z) of the lane's rows
  int32_t* dcm = reinterpret_cast<int32_t*>(smem + align16(sizeof(double) * band_lds_doubles(B)));  // [B]
  int32_t* flag = dcm + B;

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
  for (int t = tid; t < B; t += B) dcm[t] = -1;
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

  // ---- the lane's step t: columns ch, dis, ene (v = 0, 1, 2), SOE row t+1, DCM row -- all in VGPRs
  const int t = tid;
  const bool val = t < T;
  double x[3], xa[3], hi[3];
  double cch = 0.0, cdi = 0.0, loe = 0.0;  // objective of ch / dis, lower bound of ene
  double ks[4] = {0.0, 0.0, 0.0, 0.0};     // SOE row: coefficients of ch_t, dis_t, ene_t, ene_{t+1}
  double kd[3] = {0.0, 0.0, 0.0};          // DCM row: coefficients of ch_t, dis_t, tau_j
  double kp = 0.0;                         // coefficient of ene_t in row t (init row or SOE row of step t-1)
  double ys = 0.0, yas = 0.0, qsr = 0.0, yd = 0.0, yad = 0.0, qd = 0.0;
  int drow = -1, jt = 0;
#pragma unroll
  for (int v = 0; v < 3; ++v) x[v] = xa[v] = hi[v] = 0.0;
  if (val) {
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      hi[v] = us[v * T + t];
      x[v] = xa[v] = fmin(fmax(0.0, ls[v * T + t]), hi[v]);
    }
    cch = cs[t];
    cdi = cs[T + t];
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
    qsr = qs[t + 1];
    const int dv = dcm[t];
    if (dv >= 0) {
      drow = dv >> 3;
      jt = dv & 7;
      for (int p = gkp[drow]; p < gkp[drow + 1]; ++p) {
        const int c = gkc[p];
        const double a = gkv[p];
        if (c < T) kd[0] = a;
        else if (c < 2 * T) kd[1] = a;
        else kd[2] = a;
      }
      qd = qs[drow];
    }
  }
  const int xta = lds_addr(XT + jt);
  if (tid < kJMax) {  // tau columns
    const bool tv = tid < J;
    const double l0 = tv ? ls[3 * T + tid] : 0.0, h0 = tv ? us[3 * T + tid] : 0.0, x0 = fmin(fmax(0.0, l0), h0);
    TS[tid] = TS[kJMax + tid] = TS[5 * kJMax + tid] = x0;
    TS[2 * kJMax + tid] = tv ? cs[3 * T + tid] : 0.0;
    TS[3 * kJMax + tid] = l0;
    TS[4 * kJMax + tid] = h0;
    XT[tid] = 0.0;
  }
  if (tid == 0) {  // init row
    I0[0] = I0[1] = I0[2] = 0.0;
    I0[3] = qs[0];
    I0[4] = gkv[gkp[0]];
    XE[B] = YS[B] = 0.0;
  }
  XE[tid] = YS[tid] = 0.0;
  for (int u = tid; u < kJMax * B; u += B) TP[u] = 0.0;
#pragma unroll
  for (int v = 0; v < 3; ++v) XP[v * B + tid] = x[v];
  YP[tid] = YP[B + tid] = 0.0;
  __syncthreads();

  // ---- SpMV pieces (fixed summation order)
  // K^T of the lane's columns from its rows' values (vs: SOE row, vd: DCM row) and vprev = value of row t
  auto ktr = [&](double vs, double vd, double vprev, double (&out)[3]) {
    out[0] = fma(kd[0], vd, ks[0] * vs);
    out[1] = fma(kd[1], vd, ks[1] * vs);
    out[2] = fma(ks[2], vs, kp * vprev);
  };
  // K of the lane's rows, own-column part (the neighbour's ene and the tau term are added by kfin)
  auto kown = [&](const double (&v)[3], double& os, double& od) {
    os = fma(ks[2], v[2], fma(ks[1], v[1], ks[0] * v[0]));
    od = fma(kd[1], v[1], kd[0] * v[0]);
  };
  auto kfin = [&](double& os, double& od, double vnext) {
    os = fma(ks[3], vnext, os);
    od = fma(kd[2], lds_ld(xta), od);
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
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int r = 0; r < NW; r += 2) {
        a0 += TP[j * B + r * kWave + lane];
        if (r + 1 < NW) a1 += TP[j * B + (r + 1) * kWave + lane];
      }
      const double a = uniform(wave_sum_dpp(a0 + a1));
      if (lane == j) res = a;
    }
    return res;
  };

  // ---- ||Kt||_2 by power iteration (as the ELL kernel: v <- Kt'(Kt v), sigma^2 = |v_P| / |v_{P-1}|)
  double eta = scal[0];
  if (o.power_iters > 0) {
    const int P = o.power_iters;
    const double v0 = 1.0 / sqrt((double)n);
    double vc[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) vc[v] = val ? v0 : 0.0;
    double vtau = (wid == 0 && lane < J) ? v0 : 0.0;
    double nv[2] = {0.0, 0.0};
    double ws = 0.0, wd = 0.0;
    for (int pi = 0; pi <= P; ++pi) {
      if (pi > 0) {
        ktr(ws, wd, YS[tid], vc);
        if (wid == 0) {
          const double kt = tau_kt();
          vtau = lane < J ? kt : 0.0;
        }
      }
      if (pi >= P - 1) nv[pi - (P - 1)] = fma(vtau, vtau, fma(vc[2], vc[2], fma(vc[1], vc[1], vc[0] * vc[0])));
      if (pi == P) break;
      XE[tid] = vc[2];
      if (wid == 0 && lane < J) XT[lane] = vtau;
      __syncthreads();
      kown(vc, ws, wd);
      kfin(ws, wd, XE[tid + 1]);
      YS[tid + 1] = ws;
      if (tid == 0) YS[0] = I0[4] * vc[2];
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

  double mv0, mv1, mv2, mv3;
  auto iterate = [&](auto chk_tag) __attribute__((always_inline)) {
    constexpr bool CHECK = decltype(chk_tag)::value;
    if (kin - kbase >= kWave) {
      kbase = kin;
      hw = hload(kin);
    }
    const double cb = readlane_f64(hw, kin - kbase), ca = 1.0 - cb;
    mv0 = mv1 = mv2 = mv3 = 0.0;
    // ---------------- primal half-step (reflected Halpern, rho = 1)
    double kxs, kxd;  // own-column part of K x-bar for the dual half-step
    {
      double kty[3], xb[3];
      ktr(ys, yd, YS[tid], kty);
      const double cv[3] = {cch, cdi, 0.0};
      const double lv[3] = {0.0, 0.0, loe};
#pragma unroll
      for (int v = 0; v < 3; ++v) {  // branch-free: padding steps have c = lo = hi = 0 and stay at 0
        const double p1 = vmin(vmax(fma(-tau, cv[v] - kty[v], x[v]), lv[v]), hi[v]);
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
      kown(xb, kxs, kxd);
      if (wid == 0 && J > 0) {  // tau columns: K'y summed from the DCM rows' per-lane partials
        const double kt = tau_kt();
        if (lane < J) {
          const double xo = TS[lane], xan = TS[kJMax + lane];
          const double p1 = vmin(vmax(fma(-tau, TS[2 * kJMax + lane] - kt, xo), TS[3 * kJMax + lane]),
                                 TS[4 * kJMax + lane]);
          const double xbt = fma(2.0, p1, -xo);
          XT[lane] = xbt;
          TS[lane] = fma(ca, xbt, cb * xan);
          if (CHECK) {
            const double d = xo - p1, da = p1 - xan;
            mv0 += d * d;
            mv1 += da * da;
            TS[5 * kJMax + lane] = p1;
          }
        }
      }
    }
    lds_barrier();
    // ---------------- dual half-step
    {
      kfin(kxs, kxd, XE[tid + 1]);
      const double p1 = fma(sigma, qsr - kxs, ys);               // SOE row: equality
      const double p2 = vmax(fma(sigma, qd - kxd, yd), 0.0);    // DCM row: >=, its dual stays >= 0
      if (CHECK) {
        const double d = ys - p1, da = p1 - yas, e = yd - p2, ea = p2 - yad;
        mv2 += d * d + e * e;
        mv3 += da * da + ea * ea;
        YP[tid] = p1;
        YP[B + tid] = p2;
      }
      ys = fma(ca, fma(2.0, p1, -ys), cb * yas);
      yd = fma(ca, fma(2.0, p2, -yd), cb * yad);
      YS[tid + 1] = ys;
      if (J > 0) tau_parts(yd);
      if (tid == 0) {  // init row: ene_0 = target
        const double y0 = I0[0], ya0 = I0[1];
        const double q1 = fma(sigma, I0[3] - I0[4] * XE[0], y0);
        if (CHECK) {
          const double d = y0 - q1, da = q1 - ya0;
          mv2 += d * d;
          mv3 += da * da;
          I0[2] = q1;
        }
        const double yn = fma(ca, fma(2.0, q1, -y0), cb * ya0);
        I0[0] = yn;
        YS[0] = yn;
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
      iterate(F());
      continue;
    }
    ck = chk;
    iterate(Tt());
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
      double xp[3];
#pragma unroll
      for (int v = 0; v < 3; ++v) xp[v] = XP[v * B + tid];
      const double yps = YP[tid], ypd = YP[B + tid];
      XE[tid] = xp[2];
      YS[tid + 1] = yps;
      if (tid == 0) YS[0] = I0[2];
      if (wid == 0 && lane < J) XT[lane] = TS[5 * kJMax + lane];
      if (J > 0) tau_parts(ypd);
      lds_barrier();
      auto col_kkt = [&](int j, double kt, double cj, double loj, double hij, double xj) {
        loj = opaque(loj);
        hij = opaque(hij);
        const double d = dcv[opaque(j)];
        const double rc = (cj - kt) / d;
        const bool fl = isfinite(loj), fh = isfinite(hij);
        const double lam = (fl && fh) ? rc : (fl ? fmax(rc, 0.0) : (fh ? fmin(rc, 0.0) : 0.0));
        const double rd = rc - lam;
        acc[5] += rd * rd;
        acc[6] += cj * xj;
        acc[8] += (fl ? loj * d * fmax(lam, 0.0) : 0.0) + (fh ? hij * d * fmin(lam, 0.0) : 0.0);
      };
      auto row_kkt = [&](int i, double kv, double qi, double yi, bool ge) {
        double r = (qi - kv) / drv[opaque(i)];
        if (ge) r = fmax(r, 0.0);
        acc[4] += r * r;
        acc[7] += qi * yi;
      };
      double kt[3];
      ktr(yps, ypd, YS[tid], kt);
      if (val) {
        col_kkt(t, kt[0], cch, 0.0, hi[0], xp[0]);
        col_kkt(T + t, kt[1], cdi, 0.0, hi[1], xp[1]);
        col_kkt(2 * T + t, kt[2], 0.0, loe, hi[2], xp[2]);
      }
      if (wid == 0 && J > 0) {
        const double ktt = tau_kt();
        if (lane < J)
          col_kkt(3 * T + lane, ktt, TS[2 * kJMax + lane], TS[3 * kJMax + lane], TS[4 * kJMax + lane],
                  TS[5 * kJMax + lane]);
      }
      double kxs, kxd;
      kown(xp, kxs, kxd);
      kfin(kxs, kxd, XE[tid + 1]);
      if (val) row_kkt(t + 1, kxs, qsr, yps, false);
      if (drow >= 0) row_kkt(drow, kxd, qd, ypd, true);
      if (tid == 0) row_kkt(0, I0[4] * xp[2], I0[3], I0[2], false);
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
      for (int v = 0; v < 3; ++v) x[v] = xa[v] = XP[v * B + tid];
      ys = yas = YP[tid];
      yd = yad = YP[B + tid];
      if (tid == 0) I0[0] = I0[1] = I0[2];
      if (wid == 0 && lane < J) TS[lane] = TS[kJMax + lane] = TS[5 * kJMax + lane];
      kin = 0;
      kbase = 0;
      hw = hload(0);
      r0 = r;
      rprev = -1.0;
    } else {
      rprev = r;
    }
    if (restart || kkt) {  // the y images must hold z again (after a restart z = T(z_k))
      YS[tid + 1] = ys;
      if (tid == 0) YS[0] = I0[0];
      if (J > 0) tau_parts(yd);
    }
    lds_barrier();
  }
  // outputs: the last check's T(z_k), unscaled
  if (val) {
#pragma unroll
    for (int v = 0; v < 3; ++v) xo_g[v * T + t] = XP[v * B + tid] * dcv[v * T + t];
    yo_g[t + 1] = YP[tid] * drv[t + 1];
    if (drow >= 0) yo_g[drow] = YP[B + tid] * drv[drow];
  }
  if (tid < J) xo_g[3 * T + tid] = TS[5 * kJMax + tid] * dcv[3 * T + tid];
  if (tid == 0) {
    yo_g[0] = I0[2] * drv[0];
    b.istats[2 * k] = status;
    b.istats[2 * k + 1] = it;
    for (int u = 0; u < 4; ++u) b.stats[4 * k + u] = fin[u];
  }
}

}  // namespace

hipError_t launch_pdhg_band(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s) {
  constexpr int B = kBandB;
  const size_t lds = band_lds_bytes(B);
  auto kern = pdhg_band_kernel<B>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(ch.count), dim3(B), lds, s, b, w, ch, o);
  return hipGetLastError();
}

}  // namespace dvh

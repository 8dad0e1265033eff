// dvh_kernels.hip -- batched restarted reflected-Halpern PDHG for DER-VET dispatch-window LPs (gfx950).
//
// Replaces the per-window ECOS/GLPK solve behind storagevet Scenario.solve_optimization
// (dervet/MicrogridScenario.py:319); algorithm restated for tests in oracle/pdlp_ref.py.
//
// Two kernels per chunk of windows, ONE WORKGROUP PER WINDOW:
//   setup_kernel : deterministic CSR transpose, Ruiz + Pock-Chambolle scaling, power iteration for ||K||_2
//   pdhg_kernel  : the whole iteration loop in one launch.  Every primal / dual component is owned by one
//                  lane and lives in VGPRs for the life of the solve; the only per-iteration traffic is the
//                  two SpMV gathers through LDS (x-bar and y images) and, when the window fits (monthly
//                  windows do), the scaled K and K^T themselves are LDS-resident too, so an iteration
//                  touches no HBM at all.  Rows with more than kLongRow entries (the DCM tau column) are
//                  reduced by a whole wave with a shuffle tree.
// All reductions are fixed-order (wave butterflies + per-wave slots summed in wave order), so results
// are bitwise reproducible run to run.
#include "dvh_device.h"

#include <math.h>
#include <stdlib.h>

#include <type_traits>

namespace dvh {

namespace {


// ------------------------------------------------------------------------------------------------
// setup kernel
// ------------------------------------------------------------------------------------------------
constexpr int kSetupB = 256;
constexpr int kEllMax = 8;   // widest ELL slice of the fast kernel

// Row reductions over a CSR matrix: short rows one per thread, long rows one per wave.
// f(e, row) -> contribution; MAXR selects max instead of sum.  out[row] = g(row, reduced).
template <bool MAXR, class F, class G>
__device__ __forceinline__ void rows_reduce(const int32_t* ptr, int rows, const int32_t* longl, int nlong,
                                            F f, G g) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int NW = kSetupB / kWave;
  for (int i = tid; i < rows; i += kSetupB) {
    const int s = ptr[i], e = ptr[i + 1];
    if (e - s > kLongRow) continue;
    double acc = 0.0;
    for (int p = s; p < e; ++p) {
      const double v = f(p, i);
      acc = MAXR ? fmax(acc, v) : acc + v;
    }
    g(i, acc);
  }
  for (int L = wid; L < nlong; L += NW) {
    const int i = longl[L];
    const int s = ptr[i], e = ptr[i + 1];
    double a4[4] = {0.0, 0.0, 0.0, 0.0};  // 4 independent chains: 4 global loads in flight per lane
    int p = s + lane;
    for (; p + 3 * kWave < e; p += 4 * kWave) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double v = f(p + u * kWave, i);
        a4[u] = MAXR ? fmax(a4[u], v) : a4[u] + v;
      }
    }
    for (; p < e; p += kWave) {
      const double v = f(p, i);
      a4[0] = MAXR ? fmax(a4[0], v) : a4[0] + v;
    }
    double acc = MAXR ? fmax(fmax(a4[0], a4[1]), fmax(a4[2], a4[3])) : (a4[0] + a4[1]) + (a4[2] + a4[3]);
    acc = MAXR ? wave_max(acc) : wave_sum(acc);
    if (lane == 0) g(i, acc);
  }
}

// MED: the listed windows of the medium tier (n or m above small_max, solved by the chain kernel, dvh_chain.hip):
// Dr / Dc stay in the global workspace instead of LDS (they do not fit), everything else as for on-chip windows.
template <bool MED>
__global__ __launch_bounds__(kSetupB) void setup_kernel(const Batch b, const Work w, const Chunk ch, const Opts o,
                                                        const int32_t* list) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ double red[(kSetupB / kWave + 1) * 4];
  __shared__ int sh_cnt[2];
  __shared__ int sh_wt[kSetupB / kWave];
  const int k = list ? list[blockIdx.x] : ch.first + (int)blockIdx.x;  // (MED: always listed)
  const int kl = k - ch.first;
  const WinOff W = win_offsets(b, ch, k);
  const int n = W.n, m = W.m, nnz = W.nnz;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int32_t* cursor = reinterpret_cast<int32_t*>(smem);  // [n + 1]
  if (!MED && (n > o.small_max || m > o.small_max)) {  // medium tier or the grid-wide large-LP path
    if (tid == 0) {
      w.scal[(int64_t)kl * kScal] = 0.0;
      w.scal[(int64_t)kl * kScal + 6] = 2.0;
    }
    return;
  }
  // 0. crossed bounds (l_j > u_j, e.g. a reliability min-SOE requirement above the battery's energy rating): the
  //    window is primal infeasible as given; reported at once (status PRIMAL_INFEASIBLE, 0 iterations), and flagged
  //    solved (scal[6] = 3) so no PDHG kernel takes it
  {
    int crossed = 0;
    for (int j = tid; j < n; j += kSetupB) crossed |= b.l[W.on + j] > b.u[W.on + j];
    if (__syncthreads_or(crossed)) {
      if (tid == 0) {
        w.scal[(int64_t)kl * kScal] = 0.0;
        w.scal[(int64_t)kl * kScal + 6] = 3.0;
        b.istats[2 * k] = 1;  // DVH_PRIMAL_INFEASIBLE
        b.istats[2 * k + 1] = 0;
        for (int u = 0; u < 4; ++u) b.stats[4 * k + u] = u == 0 ? NAN : 0.0;
      }
      return;
    }
  }

  const int32_t* Kp = b.indptr + W.row;
  const int32_t* Kc = b.indices + W.nz;
  const double* Kv = b.data + W.nz;
  int32_t* Tp = w.tptr + W.wtr;
  int32_t* Ti = w.tind + W.wz;
  double* Tv = w.tval + W.wz;
  double* KV = w.kval + W.wz;
  int32_t* rowof = w.rowof + W.wz;
  int32_t* perm = w.perm + W.wz;
  double* gDr = w.dr + W.wm;
  double* gDc = w.dc + W.wn;
  double* tmpr = w.tmpr + W.wm;
  double* tmpc = w.tmpc + W.wn;
  int32_t* longk = w.longk + (int64_t)kl * kLMax;
  int32_t* longt = w.longt + (int64_t)kl * kLMax;
  double* scal = w.scal + (int64_t)kl * kScal;

  // 1. entry -> row map; per-segment column counts (the nnz are split into nseg contiguous segments, one
  //    wave each; counts are order-independent, so the layout below is deterministic)
  const int nseg = o.setup_segments;
  for (int j = tid; j < nseg * (n + 1); j += kSetupB) cursor[j] = 0;
  __syncthreads();
  for (int i = tid; i < m; i += kSetupB)
    for (int p = Kp[i]; p < Kp[i + 1]; ++p) rowof[p] = i;
  auto seg_lo = [&](int sg) { return (int)(((long long)nnz * sg) / nseg); };
  for (int sg = 0; sg < nseg; ++sg) {
    const int a = seg_lo(sg), e = seg_lo(sg + 1);
    for (int p = a + tid; p < e; p += kSetupB) atomicAdd(&cursor[sg * (n + 1) + Kc[p]], 1);
  }
  __syncthreads();
  // 2. column totals, exclusive scan -> Tp; per-segment cursors = Tp + counts of earlier segments
  {
    const int per = (n + kSetupB - 1) / kSetupB;
    const int s0 = tid * per, e0 = min(n, s0 + per);
    int acc = 0;
    for (int j = s0; j < e0; ++j)
      for (int sg = 0; sg < nseg; ++sg) acc += cursor[sg * (n + 1) + j];
    // exclusive scan of the per-thread totals (integer: exact in any order): wave scans, then the wave totals
    int inc = acc;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int t = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += t;
    }
    if (lane == kWave - 1) sh_wt[wid] = inc;
    __syncthreads();
    int run = inc - acc;
    for (int u = 0; u < wid; ++u) run += sh_wt[u];
    for (int j = s0; j < e0; ++j) {
      Tp[j] = run;
      for (int sg = 0; sg < nseg; ++sg) {
        const int v = cursor[sg * (n + 1) + j];
        cursor[sg * (n + 1) + j] = run;
        run += v;
      }
    }
    if (tid == 0) Tp[n] = nnz;
  }
  __syncthreads();
  // 3. stable fill of K^T, wave sg walks segment sg in row-major order; ties inside a 64-entry chunk are
  //    ranked by lane
  if (wid < nseg) {
    const int nb = 32 - __builtin_clz((unsigned)(n > kWave ? n : kWave));
    int32_t* cur = cursor + wid * (n + 1);
    const int a = seg_lo(wid), e = seg_lo(wid + 1);
    for (int base = a; base < e; base += kWave) {
      const int p = base + lane;
      const bool v = p < e;
      const int j = v ? Kc[p] : -1 - lane;
      // lanes holding the same column: AND of one ballot per bit of j (bits 0 .. nb-1 cover the columns and the
      // padding lanes' -1 - lane among themselves; the sign bit tells the two apart)
      unsigned long long eq = ~0ull;
      for (int bt = 0; bt < nb; ++bt) {
        const bool on = (j >> bt) & 1;
        const unsigned long long bal = __ballot(on);
        eq &= on ? bal : ~bal;
      }
      {
        const bool on = j < 0;
        const unsigned long long bal = __ballot(on);
        eq &= on ? bal : ~bal;
      }
      const int rank = __popcll(eq & ((1ull << lane) - 1ull)), cnt = __popcll(eq);
      int pos = 0;
      if (v) pos = cur[j] + rank;
      __builtin_amdgcn_wave_barrier();
      if (v) {
        Ti[pos] = rowof[p];
        Tv[pos] = Kv[p];
        perm[p] = pos;
        if (rank == cnt - 1) cur[j] = pos + 1;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  __syncthreads();
  // 4. long-row lists (deterministic ballot compaction): every thread flags rows / columns (bytes over the dead
  //    transpose cursors), wave 0 compacts the flags from LDS
  unsigned char* lfl = reinterpret_cast<unsigned char*>(cursor);
  // (the cursors hold nseg (n + 1) ints; a window with more rows than that reads the lengths from global memory)
  const bool fl_lds = (int64_t)m + n <= 4 * (int64_t)nseg * (n + 1);
  auto row_long = [&](int i) { return fl_lds ? lfl[i] != 0 : (Kp[i + 1] - Kp[i]) > kLongRow; };
  auto col_long = [&](int j) { return fl_lds ? lfl[m + j] != 0 : (Tp[j + 1] - Tp[j]) > kLongRow; };
  if (fl_lds) {
    for (int i = tid; i < m; i += kSetupB) lfl[i] = (Kp[i + 1] - Kp[i]) > kLongRow;
    for (int j = tid; j < n; j += kSetupB) lfl[m + j] = (Tp[j + 1] - Tp[j]) > kLongRow;
  }
  __syncthreads();
  if (wid == 0) {
    int nk = 0, nt = 0;
    for (int base = 0; base < m; base += kWave) {
      const int i = base + lane;
      const bool isl = i < m && row_long(i);
      const unsigned long long bal = __ballot(isl);
      const int pre = __popcll(bal & ((1ull << lane) - 1ull));
      if (isl && nk + pre < kLMax) longk[nk + pre] = i;
      nk += __popcll(bal);
    }
    for (int base = 0; base < n; base += kWave) {
      const int j = base + lane;
      const bool isl = j < n && col_long(j);
      const unsigned long long bal = __ballot(isl);
      const int pre = __popcll(bal & ((1ull << lane) - 1ull));
      if (isl && nt + pre < kLMax) longt[nt + pre] = j;
      nt += __popcll(bal);
    }
    if (lane == 0) {
      sh_cnt[0] = nk;
      sh_cnt[1] = nt;
    }
  }
  __syncthreads();
  const int nlk = sh_cnt[0], nlt = sh_cnt[1];
  if (nlk > kLMax || nlt > kLMax) {  // unsupported structure: more dense rows than the on-chip lists
    if (tid == 0) {
      scal[0] = 0.0;
      scal[6] = 1.0;
    }
    return;
  }
  // 5. Ruiz (inf-norm) passes, then one Pock-Chambolle (alpha = 1) pass.  Dr / Dc live in LDS from here on
  //    (the transpose cursors are dead): the row / column passes gather Dc[Kc[p]] and Dr[Ti[p]] from LDS
  //    instead of a dependent global load; copied to the workspace at the end.
  double* Dr = MED ? gDr : reinterpret_cast<double*>(smem);
  double* Dc = MED ? gDc : Dr + m;
  for (int j = tid; j < n; j += kSetupB) Dc[j] = 1.0;
  for (int i = tid; i < m; i += kSetupB) Dr[i] = 1.0;
  __syncthreads();
  for (int pass = 0; pass <= o.ruiz_iters; ++pass) {
    const bool pc = pass == o.ruiz_iters;
    auto fr = [&](int p, int i) { return fabs(Kv[p]) * Dr[i] * Dc[Kc[p]]; };
    auto gr = [&](int i, double a) { tmpr[i] = a > 0.0 ? 1.0 / sqrt(a) : 1.0; };
    auto fc = [&](int p, int j) { return fabs(Tv[p]) * Dc[j] * Dr[Ti[p]]; };
    auto gc = [&](int j, double a) { tmpc[j] = a > 0.0 ? 1.0 / sqrt(a) : 1.0; };
    if (pc) {
      rows_reduce<false>(Kp, m, longk, nlk, fr, gr);
      rows_reduce<false>(Tp, n, longt, nlt, fc, gc);
    } else {
      rows_reduce<true>(Kp, m, longk, nlk, fr, gr);
      rows_reduce<true>(Tp, n, longt, nlt, fc, gc);
    }
    __syncthreads();
    int changed = 0;
    for (int j = tid; j < n; j += kSetupB) {
      const double t = tmpc[j];
      changed |= t != 1.0;
      Dc[j] *= t;
    }
    for (int i = tid; i < m; i += kSetupB) {
      const double t = tmpr[i];
      changed |= t != 1.0;
      Dr[i] *= t;
    }
    // A Ruiz pass whose factors are all exactly 1 left Dr / Dc unchanged, so every further Ruiz pass would
    // repeat it bit for bit: skip to the Pock-Chambolle pass (same result, fewer passes).
    if (__syncthreads_or(changed) == 0 && !pc) pass = o.ruiz_iters - 1;
  }
  // 6. scaled data
  for (int p = tid; p < nnz; p += kSetupB) {
    const double v = Kv[p] * Dr[rowof[p]] * Dc[Kc[p]];
    KV[p] = v;
    Tv[perm[p]] = v;
  }
  double nrm[4] = {0.0, 0.0, 0.0, 0.0};  // ||cs||^2, ||qs||^2, ||c||^2, ||q||^2
  for (int j = tid; j < n; j += kSetupB) {
    const double cj = b.c[W.on + j], d = Dc[j];
    w.cs[W.wn + j] = cj * d;
    w.ls[W.wn + j] = b.l[W.on + j] / d;
    w.us[W.wn + j] = b.u[W.on + j] / d;
    nrm[0] += cj * d * cj * d;
    nrm[2] += cj * cj;
  }
  for (int i = tid; i < m; i += kSetupB) {
    const double qi = b.q[W.om + i], d = Dr[i];
    w.qs[W.wm + i] = qi * d;
    nrm[1] += qi * d * qi * d;
    nrm[3] += qi * qi;
  }
  // (the single-precision factor copies Work::fc / fr are the band kernels' own: they scale their windows themselves
  // and never run after this kernel, so none are written here)
  if (!MED) {
    for (int j = tid; j < n; j += kSetupB) gDc[j] = Dc[j];
    for (int i = tid; i < m; i += kSetupB) gDr[i] = Dr[i];
  }
  block_sum<kSetupB, 4>(nrm, red);
  // 8. row-length statistics for the ELL fast path: max length among rows with <= kEllMax entries and
  //    the number of longer rows, for K and K^T
  double wst[4] = {0.0, 0.0, 0.0, 0.0};
  for (int i = tid; i < m; i += kSetupB) {
    const int len = Kp[i + 1] - Kp[i];
    if (len <= kEllMax) wst[0] = fmax(wst[0], (double)len); else wst[2] += 1.0;
  }
  for (int j = tid; j < n; j += kSetupB) {
    const int len = Tp[j + 1] - Tp[j];
    if (len <= kEllMax) wst[1] = fmax(wst[1], (double)len); else wst[3] += 1.0;
  }
  {
    double mx[2] = {wave_max(wst[0]), wave_max(wst[1])};
    double ct[2] = {wst[2], wst[3]};
    block_sum<kSetupB, 2>(ct, red);
    if (lane == 0) { red[wid * 2] = mx[0]; red[wid * 2 + 1] = mx[1]; }
    __syncthreads();
    if (tid == 0) {
      double a = 0.0, c2 = 0.0;
      for (int t = 0; t < kSetupB / kWave; ++t) { a = fmax(a, red[2 * t]); c2 = fmax(c2, red[2 * t + 1]); }
      scal[8] = a;
      scal[9] = c2;
      scal[10] = ct[0];
      scal[11] = ct[1];
    }
  }
  if (tid == 0) {
    const double ncs = sqrt(nrm[0]), nqs = sqrt(nrm[1]);
    scal[0] = o.step_safety;  // Pock-Chambolle bound ||Kt|| <= 1; the PDHG kernels refine it (power iteration)
    scal[1] = (ncs > 1e-10 && nqs > 1e-10) ? ncs / nqs : 1.0;
    scal[2] = sqrt(nrm[2]);
    scal[3] = sqrt(nrm[3]);
    scal[4] = (double)nlk;
    scal[5] = (double)nlt;
    scal[6] = 0.0;
    scal[7] = 1.0;
  }
}

// Power iteration on Kt'Kt for the windows of the generic path (the ELL kernel runs its own on chip).
__global__ __launch_bounds__(kSetupB) void power_kernel(const Batch b, const Work w, const Chunk ch, const Opts o,
                                                        const int32_t* list) {
  __shared__ double red[(kSetupB / kWave + 1) * 4];
  const int k = list[blockIdx.x];
  const int kl = k - ch.first;
  const WinOff W = win_offsets(b, ch, k);
  const int n = W.n, m = W.m;
  const int tid = threadIdx.x;
  const int32_t* Kp = b.indptr + W.row;
  const int32_t* Kc = b.indices + W.nz;
  const int32_t* Tp = w.tptr + W.wtr;
  const int32_t* Ti = w.tind + W.wz;
  const double* Tv = w.tval + W.wz;
  const double* KV = w.kval + W.wz;
  double* tmpc = w.tmpc + W.wn;
  const int32_t* longk = w.longk + (int64_t)kl * kLMax;
  const int32_t* longt = w.longt + (int64_t)kl * kLMax;
  double* scal = w.scal + (int64_t)kl * kScal;
  if (scal[6] != 0.0 || o.power_iters <= 0) return;
  const int nlk = (int)scal[4], nlt = (int)scal[5];
  double* v = w.vbuf + W.wn;
  double* wv = w.wbuf + W.wm;
  const double v0 = 1.0 / sqrt((double)(n > 0 ? n : 1));
  for (int j = tid; j < n; j += kSetupB) v[j] = v0;
  __syncthreads();
  double sig = 0.0;
  for (int it = 0; it < o.power_iters; ++it) {
    rows_reduce<false>(Kp, m, longk, nlk, [&](int p, int) { return KV[p] * v[Kc[p]]; },
                       [&](int i, double a) { wv[i] = a; });
    __syncthreads();
    double s2[1] = {0.0};
    rows_reduce<false>(Tp, n, longt, nlt, [&](int p, int) { return Tv[p] * wv[Ti[p]]; },
                       [&](int j, double a) { tmpc[j] = a; });
    __syncthreads();
    for (int j = tid; j < n; j += kSetupB) s2[0] += tmpc[j] * tmpc[j];
    block_sum<kSetupB, 1>(s2, red);
    const double nv = sqrt(s2[0]);
    sig = sqrt(nv);
    const double inv = nv > 0.0 ? 1.0 / nv : 0.0;
    for (int j = tid; j < n; j += kSetupB) v[j] = tmpc[j] * inv;
    __syncthreads();
  }
  if (tid == 0 && sig > 0.0) {
    scal[0] = o.step_safety / sig;
    scal[7] = sig;
  }
}

// ------------------------------------------------------------------------------------------------
// PDHG kernel
// ------------------------------------------------------------------------------------------------

template <bool MLDS>
struct MatView;

template <>
struct MatView<true> {  // LDS-resident scaled matrices (16-bit column indices)
  const int32_t* kp;
  const uint16_t* kc;
  const double* kv;
  const int32_t* tp;
  const uint16_t* tc;
  const double* tv;
};
template <>
struct MatView<false> {  // matrices read from the workspace (L2 / Infinity Cache)
  const int32_t* kp;
  const int32_t* kc;
  const double* kv;
  const int32_t* tp;
  const int32_t* tc;
  const double* tv;
};


// LDS bytes needed by the PDHG kernel for a window (layout in pdhg_kernel).
__host__ __device__ inline size_t pdhg_lds_bytes(int n, int m, int nnz, bool mlds, int nwaves) {
  size_t s = align16(sizeof(double) * ((size_t)n + m + (size_t)kNRed * (nwaves + 1) + 10 * kLMax));
  s += align16(sizeof(int32_t) * 2 * kLMax);
  if (mlds) {
    s += align16(sizeof(double) * 2 * (size_t)nnz);
    s += align16(sizeof(int32_t) * ((size_t)n + m + 2));
    s += align16(sizeof(uint16_t) * 2 * (size_t)nnz);
  }
  return s;
}

template <int B, int XS, int YS, bool MLDS>
__global__ __launch_bounds__(B) void pdhg_kernel(const Batch b, const Work w, const Chunk ch, const Opts o,
                                                 const int32_t* list) {
  constexpr int NW = B / kWave;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int k = list ? list[blockIdx.x] : ch.first + blockIdx.x;
  const int kl = k - ch.first;
  const WinOff W = win_offsets(b, ch, k);
  const int n = W.n, m = W.m, meq = W.meq, nnz = W.nnz;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const double* scal = w.scal + (int64_t)kl * kScal;
  const int nlk = (int)scal[4], nlt = (int)scal[5];
  if (scal[6] == 3.0) return;  // reported infeasible by the setup kernel
  if (scal[6] != 0.0 || n > XS * B || m > YS * B || (MLDS && (n > 65535 || m > 65535))) {
    if (tid == 0) {
      b.istats[2 * k] = kNumerical;
      b.istats[2 * k + 1] = 0;
      for (int t = 0; t < 4; ++t) b.stats[4 * k + t] = NAN;
    }
    return;
  }
  // ---- LDS carve (all double arrays first, 16-byte aligned sections)
  double* X = reinterpret_cast<double*>(smem);
  double* Y = X + n;
  double* red = Y + m;
  double* lx = red + kNRed * (NW + 1);  // long columns: x, xa, c, lo, hi, xp   [6][kLMax]
  double* ly = lx + 6 * kLMax;          // long rows:    y, ya, q, yp           [4][kLMax]
  unsigned char* cur = smem + align16(sizeof(double) * ((size_t)n + m + (size_t)kNRed * (NW + 1) + 10 * kLMax));
  int32_t* lxi = reinterpret_cast<int32_t*>(cur);
  int32_t* lyi = lxi + kLMax;
  cur += align16(sizeof(int32_t) * 2 * kLMax);
  MatView<MLDS> M;
  if constexpr (MLDS) {
    double* kv = reinterpret_cast<double*>(cur);
    double* tv = kv + nnz;
    cur += align16(sizeof(double) * 2 * (size_t)nnz);
    int32_t* kp = reinterpret_cast<int32_t*>(cur);
    int32_t* tp = kp + (m + 1);
    cur += align16(sizeof(int32_t) * ((size_t)n + m + 2));
    uint16_t* kc = reinterpret_cast<uint16_t*>(cur);
    uint16_t* tc = kc + nnz;
    const int32_t* gkp = b.indptr + W.row;
    const int32_t* gkc = b.indices + W.nz;
    const int32_t* gtp = w.tptr + W.wtr;
    const int32_t* gtc = w.tind + W.wz;
    const double* gkv = w.kval + W.wz;
    const double* gtv = w.tval + W.wz;
    for (int p = tid; p < nnz; p += B) {
      kv[p] = gkv[p];
      tv[p] = gtv[p];
      kc[p] = (uint16_t)gkc[p];
      tc[p] = (uint16_t)gtc[p];
    }
    for (int i = tid; i <= m; i += B) kp[i] = gkp[i];
    for (int j = tid; j <= n; j += B) tp[j] = gtp[j];
    M.kp = kp; M.kc = kc; M.kv = kv; M.tp = tp; M.tc = tc; M.tv = tv;
  } else {
    M.kp = b.indptr + W.row;
    M.kc = b.indices + W.nz;
    M.kv = w.kval + W.wz;
    M.tp = w.tptr + W.wtr;
    M.tc = w.tind + W.wz;
    M.tv = w.tval + W.wz;
  }
  const int32_t* glk = w.longk + (int64_t)kl * kLMax;
  const int32_t* glt = w.longt + (int64_t)kl * kLMax;
  const double* cs = w.cs + W.wn;
  const double* ls = w.ls + W.wn;
  const double* us = w.us + W.wn;
  const double* qs = w.qs + W.wm;
  const double* dcv = w.dc + W.wn;
  const double* drv = w.dr + W.wm;
  for (int L = tid; L < nlt; L += B) {
    const int j = glt[L];
    lxi[L] = j;
    const double lo = ls[j], hi = us[j];
    const double x0 = fmin(fmax(0.0, lo), hi);
    lx[0 * kLMax + L] = x0;
    lx[1 * kLMax + L] = x0;
    lx[2 * kLMax + L] = cs[j];
    lx[3 * kLMax + L] = lo;
    lx[4 * kLMax + L] = hi;
    lx[5 * kLMax + L] = x0;
  }
  for (int L = tid; L < nlk; L += B) {
    const int i = glk[L];
    lyi[L] = i;
    ly[0 * kLMax + L] = 0.0;
    ly[1 * kLMax + L] = 0.0;
    ly[2 * kLMax + L] = qs[i];
    ly[3 * kLMax + L] = 0.0;
  }
  __syncthreads();

  // ---- register-resident state of the lane-owned (short) columns and rows
  double x[XS], xa[XS], cc[XS], lo[XS], hi[XS];
  double* xo_g = b.x + W.on;  // x+ (scaled) at check iterations, final unscaled x
  double* yo_g = b.y + W.om;
  int ts[XS], te[XS];
#pragma unroll
  for (int s = 0; s < XS; ++s) {
    const int j = tid + s * B;
    ts[s] = te[s] = 0;
    x[s] = xa[s] = cc[s] = lo[s] = hi[s] = 0.0;
    if (j < n) {
      const int a0 = M.tp[j], a1 = M.tp[j + 1];
      if (a1 - a0 <= kLongRow) {
        ts[s] = a0;
        te[s] = a1;
        cc[s] = cs[j];
        lo[s] = ls[j];
        hi[s] = us[j];
        x[s] = xa[s] = fmin(fmax(0.0, lo[s]), hi[s]);
        xo_g[j] = x[s];
      } else {
        ts[s] = te[s] = -1;  // long column: owned by a wave
      }
    } else {
      ts[s] = te[s] = -1;
    }
  }
  double y[YS], ya[YS], qq[YS];
  int ks[YS], ke[YS];
#pragma unroll
  for (int s = 0; s < YS; ++s) {
    const int i = tid + s * B;
    y[s] = ya[s] = qq[s] = 0.0;
    ks[s] = ke[s] = -1;
    if (i < m) {
      const int a0 = M.kp[i], a1 = M.kp[i + 1];
      if (a1 - a0 <= kLongRow) {
        ks[s] = a0;
        ke[s] = a1;
        qq[s] = qs[i];
        yo_g[i] = 0.0;
      }
      Y[i] = 0.0;
    }
  }
  __syncthreads();

  double eta = scal[0], pw = scal[1];
  const double cnorm = scal[2], qnorm = scal[3], c0 = b.c0[k];
  const double rho = o.rho;
  int it = 0, kin = 0, status = kIterLimit;
  double r0 = -1.0, rprev = -1.0;
  double fin[4] = {NAN, NAN, NAN, NAN};  // obj, pres, dres, gap at the last check
  const int chk = o.check_every > 0 ? o.check_every : 64;
  const int kkt_every = o.kkt_every > 0 ? o.kkt_every : 1;
  int ck = chk, kk = kkt_every;

  while (it < o.max_iters) {
    const double tau = eta / pw, sigma = eta * pw;
    const bool check = --ck == 0;
    if (check) ck = chk;
    // Halpern weights: 1/(k+2) from the host table (uniform index -> scalar load), exact quotient beyond it
    const double cb = kin < kHalpernTab ? w.hinv[kin] : 1.0 / (kin + 2.0), ca = 1.0 - cb;
    double acc[kNRed];
#pragma unroll
    for (int t = 0; t < kNRed; ++t) acc[t] = 0.0;
    // ---------------- primal half-step: x+ = proj(x - tau (c - K'y)), X <- 2x+ - x
#pragma unroll
    for (int s = 0; s < XS; ++s) {
      if (ts[s] >= 0) {
        const int j = tid + s * B;
        double kty = 0.0;
        for (int p = ts[s]; p < te[s]; ++p) kty += M.tv[p] * Y[M.tc[p]];
        const double p1 = fmin(fmax(x[s] - tau * (cc[s] - kty), lo[s]), hi[s]);
        X[j] = 2.0 * p1 - x[s];
        if (check) {
          const double d = x[s] - p1, da = p1 - xa[s];
          acc[0] += d * d;
          acc[1] += da * da;
          xo_g[j] = p1;
        }
        x[s] = ca * ((1.0 + rho) * p1 - rho * x[s]) + cb * xa[s];
      }
    }
    for (int L = wid; L < nlt; L += NW) {
      const int j = lxi[L];
      double kty = 0.0;
      for (int p = M.tp[j] + lane; p < M.tp[j + 1]; p += kWave) kty += M.tv[p] * Y[M.tc[p]];
      kty = wave_sum(kty);
      if (lane == 0) {
        const double xo = lx[L], xan = lx[kLMax + L];
        const double p1 = fmin(fmax(xo - tau * (lx[2 * kLMax + L] - kty), lx[3 * kLMax + L]), lx[4 * kLMax + L]);
        X[j] = 2.0 * p1 - xo;
        if (check) {
          const double d = xo - p1, da = p1 - xan;
          acc[0] += d * d;
          acc[1] += da * da;
          lx[5 * kLMax + L] = p1;
        }
        lx[L] = ca * ((1.0 + rho) * p1 - rho * xo) + cb * xan;
      }
    }
    __syncthreads();
    // ---------------- dual half-step: y+ = proj(y + sigma (q - K X)); Y <- Halpern(y)
#pragma unroll
    for (int s = 0; s < YS; ++s) {
      if (ks[s] >= 0) {
        const int i = tid + s * B;
        double kx = 0.0;
        for (int p = ks[s]; p < ke[s]; ++p) kx += M.kv[p] * X[M.kc[p]];
        double p1 = y[s] + sigma * (qq[s] - kx);
        if (i >= meq) p1 = fmax(p1, 0.0);
        if (check) {
          const double d = y[s] - p1, da = p1 - ya[s];
          acc[2] += d * d;
          acc[3] += da * da;
          yo_g[i] = p1;
        }
        y[s] = ca * ((1.0 + rho) * p1 - rho * y[s]) + cb * ya[s];
        Y[i] = y[s];
      }
    }
    for (int L = wid; L < nlk; L += NW) {
      const int i = lyi[L];
      double kx = 0.0;
      for (int p = M.kp[i] + lane; p < M.kp[i + 1]; p += kWave) kx += M.kv[p] * X[M.kc[p]];
      kx = wave_sum(kx);
      if (lane == 0) {
        const double yo = ly[L], yan = ly[kLMax + L];
        double p1 = yo + sigma * (ly[2 * kLMax + L] - kx);
        if (i >= meq) p1 = fmax(p1, 0.0);
        if (check) {
          const double d = yo - p1, da = p1 - yan;
          acc[2] += d * d;
          acc[3] += da * da;
          ly[3 * kLMax + L] = p1;
        }
        const double yn = ca * ((1.0 + rho) * p1 - rho * yo) + cb * yan;
        ly[L] = yn;
        Y[i] = yn;
      }
    }
    ++it;
    ++kin;
    __syncthreads();
    if (!check) continue;

    // ---------------- check: restart test; every kkt_every-th check also the KKT error of T(z) = (x+, y+)
    const bool kkt = (--kk == 0) || (it + chk > o.max_iters);
    if (kkt) kk = kkt_every;
    if (kkt) {
#pragma unroll
    for (int s = 0; s < XS; ++s)
      if (ts[s] >= 0) X[tid + s * B] = xo_g[tid + s * B];
#pragma unroll
    for (int s = 0; s < YS; ++s)
      if (ks[s] >= 0) Y[tid + s * B] = yo_g[tid + s * B];
    for (int L = tid; L < nlt; L += B) X[lxi[L]] = lx[5 * kLMax + L];
    for (int L = tid; L < nlk; L += B) Y[lyi[L]] = ly[3 * kLMax + L];
    __syncthreads();
    // acc[4] = ||r_p||^2, acc[5] = ||r_d||^2, acc[6] = c'x, acc[7] = q'y, acc[8] = bound term
    auto col_kkt = [&](int j, double kty, double cj, double loj, double hij, double xj) {
      const double d = dcv[j];
      const double rc = (cj - kty) / d;
      const bool fl = isfinite(loj), fh = isfinite(hij);
      const double lam = (fl && fh) ? rc : (fl ? fmax(rc, 0.0) : (fh ? fmin(rc, 0.0) : 0.0));
      const double rd = rc - lam;
      acc[5] += rd * rd;
      acc[6] += cj * xj;
      acc[8] += (fl ? loj * d * fmax(lam, 0.0) : 0.0) + (fh ? hij * d * fmin(lam, 0.0) : 0.0);
      if (DVH_KKT_RDX) acc[kRdx] += fabs(rd) * fabs(xj * d);
    };
    auto row_kkt = [&](int i, double kx, double qi, double yi) {
      const double d = drv[i];
      double r = (qi - kx) / d;
      if (i >= meq) r = fmax(r, 0.0);
      acc[4] += r * r;
      acc[7] += qi * yi;
      acc[9] += (yi * d) * (yi * d);
    };
#pragma unroll
    for (int s = 0; s < XS; ++s) {
      if (ts[s] >= 0) {
        double kty = 0.0;
        for (int p = ts[s]; p < te[s]; ++p) kty += M.tv[p] * Y[M.tc[p]];
        col_kkt(tid + s * B, kty, cc[s], lo[s], hi[s], X[tid + s * B]);
      }
    }
    for (int L = wid; L < nlt; L += NW) {
      const int j = lxi[L];
      double kty = 0.0;
      for (int p = M.tp[j] + lane; p < M.tp[j + 1]; p += kWave) kty += M.tv[p] * Y[M.tc[p]];
      kty = wave_sum(kty);
      if (lane == 0) col_kkt(j, kty, lx[2 * kLMax + L], lx[3 * kLMax + L], lx[4 * kLMax + L], lx[5 * kLMax + L]);
    }
#pragma unroll
    for (int s = 0; s < YS; ++s) {
      if (ks[s] >= 0) {
        double kx = 0.0;
        for (int p = ks[s]; p < ke[s]; ++p) kx += M.kv[p] * X[M.kc[p]];
        row_kkt(tid + s * B, kx, qq[s], Y[tid + s * B]);
      }
    }
    for (int L = wid; L < nlk; L += NW) {
      const int i = lyi[L];
      double kx = 0.0;
      for (int p = M.kp[i] + lane; p < M.kp[i + 1]; p += kWave) kx += M.kv[p] * X[M.kc[p]];
      kx = wave_sum(kx);
      if (lane == 0) row_kkt(i, kx, ly[2 * kLMax + L], ly[3 * kLMax + L]);
    }
    }
    block_sum<B, kNRed>(acc, red);
    if (kkt) {
      const double pobj = acc[6] + c0, dobj = acc[7] + acc[8] + c0;
      const double pres = sqrt(acc[4]) / (1.0 + qnorm), dres = sqrt(acc[5]) / (1.0 + cnorm);
      const double gap = fabs(pobj - dobj) / (1.0 + fabs(pobj) + fabs(dobj));
      fin[0] = pobj;
      fin[1] = pres;
      fin[2] = dres;
      fin[3] = gap;
      if (kkt_done(o, pres, dres, gap, pobj, dobj, acc[4], acc[9], DVH_KKT_RDX ? acc[kRdx] : 0.0)) {
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
      if (ddx > 1e-10 && ddy > 1e-10) pw = pw_update(ddy / ddx, pw, o.theta);
#pragma unroll
      for (int s = 0; s < XS; ++s)
        if (ts[s] >= 0) x[s] = xa[s] = xo_g[tid + s * B];
#pragma unroll
      for (int s = 0; s < YS; ++s)
        if (ks[s] >= 0) y[s] = ya[s] = yo_g[tid + s * B];
      for (int L = tid; L < nlt; L += B) lx[L] = lx[kLMax + L] = lx[5 * kLMax + L];
      for (int L = tid; L < nlk; L += B) ly[L] = ly[kLMax + L] = ly[3 * kLMax + L];
      // Y <- y+ (the new iterate)
#pragma unroll
      for (int s = 0; s < YS; ++s)
        if (ks[s] >= 0) Y[tid + s * B] = y[s];
      for (int L = tid; L < nlk; L += B) Y[lyi[L]] = ly[3 * kLMax + L];
      kin = 0;
      r0 = r;
      rprev = -1.0;
    } else {
      rprev = r;
      if (kkt) {
#pragma unroll
        for (int s = 0; s < YS; ++s)
          if (ks[s] >= 0) Y[tid + s * B] = y[s];
        for (int L = tid; L < nlk; L += B) Y[lyi[L]] = ly[L];
      }
    }
    __syncthreads();
  }
  // ---- outputs: the last checked candidate T(z), unscaled
#pragma unroll
  for (int s = 0; s < XS; ++s)
    if (ts[s] >= 0) {
      const int j = tid + s * B;
      xo_g[j] *= dcv[j];
    }
  for (int L = tid; L < nlt; L += B) b.x[W.on + lxi[L]] = lx[5 * kLMax + L] * dcv[lxi[L]];
#pragma unroll
  for (int s = 0; s < YS; ++s)
    if (ks[s] >= 0) {
      const int i = tid + s * B;
      yo_g[i] *= drv[i];
    }
  for (int L = tid; L < nlk; L += B) b.y[W.om + lyi[L]] = ly[3 * kLMax + L] * drv[lyi[L]];
  if (tid == 0) {
    b.istats[2 * k] = status;
    b.istats[2 * k + 1] = it;
    for (int t = 0; t < 4; ++t) b.stats[4 * k + t] = fin[t];
  }
}

// ------------------------------------------------------------------------------------------------
// ELL fast-path PDHG kernel
// ------------------------------------------------------------------------------------------------
// Lane tid owns columns j = tid + s*B (s < XS) and rows i = tid + s*B (s < YS).  Short rows (K rows with
// <= WY entries, K^T rows with <= WX entries) are stored as column-major ELL slices in LDS
// (value[e][slot], coalesced ds_read_b64) with their column indices held in VGPRs for the whole solve,
// so an iteration issues every value load and gather of a lane back to back.  Long rows (the dense DCM
// tau column of K^T, or any longer row) are never gathered in the loop: their products are accumulated
// on the *producing* side -- each lane adds K_ij * y_i (or K_ij * xbar_j) of its short rows into a per-wave
// partial with a segmented wave reduction -- and one lane sums the NW partials after the barrier that
// already separates the two half-steps.  Windows that do not fit this shape are reported with
// istats status -1 and re-run by the generic kernel.
constexpr int kNeedsGeneric = -1;

// Segmented wave reduction of (target, value) pairs into part[target] (lane 0 accumulates).
__device__ __forceinline__ void wave_scatter(double v, int tgt, double* part) {
  const int lane = threadIdx.x & 63;
  unsigned long long act = __ballot(tgt >= 0);
  while (act) {
    const int leader = __ffsll((long long)act) - 1;
    const int tf = __shfl(tgt, leader, kWave);
    const bool sel = tgt == tf;
    const double sum = wave_sum_dpp(sel ? v : 0.0);
    if (lane == 0) part[tf] += sum;
    act &= ~__ballot(sel);
  }
}

// KR bit 0: the ELL values of K^T live in VGPRs (else in LDS, [WX][RX] column-major slices); bit 1: those of K
// (else [WY][RY] in LDS).  KR != 0 variants also keep T(z_k) = (x+, y+) of the last check in LDS images
// (else in the x / y output arrays in HBM).
__host__ __device__ constexpr size_t ell_lds_doubles(int n, int m, int B, int XS, int YS, int WX, int WY, int KR) {
  const int NW = B / kWave;
  const size_t img = (size_t)n + m + 2 * (size_t)B;
  return img + (KR ? img : 0) + ((KR & 1) ? 0 : (size_t)WX * XS * B) + ((KR & 2) ? 0 : (size_t)WY * YS * B) +
         2 * (size_t)NW * kLMax + (size_t)kNRed * (NW + 1) + 4 + 12 * kLMax;
}
__host__ __device__ constexpr size_t ell_lds_bytes(int n, int m, int B, int XS, int YS, int WX, int WY, int KR) {
  const size_t d = ell_lds_doubles(n, m, B, XS, YS, WX, WY, KR);
  return align16(sizeof(double) * d) + align16(sizeof(int32_t) * 4 * kLMax);
}


// WPE: minimum waves per SIMD the register allocation must allow (the small-window variants run several
// single- or two-wave workgroups per CU and need the occupancy; the large ones are sized by B alone).
// GATE: the predicted KKT gate compiled in only when dvh_options.kkt_predict > 0 (as pdhg_band_kernel: a runtime
// branch kept both check paths' state live and spilled)
template <int B, int XS, int YS, int WX, int WY, int KR, int WPE = 1, bool GATE = false>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(WPE))) void pdhg_ell_kernel(
    const Batch b, const Work w, const Chunk ch, const Opts o, const int32_t* list) {
  constexpr int NW = B / kWave;
  constexpr int RX = XS * B, RY = YS * B;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int k = list ? list[blockIdx.x] : ch.first + (int)blockIdx.x;  // list: global window ids
  const int kl = k - ch.first;
  const WinOff W = win_offsets(b, ch, k);
  const int n = W.n, m = W.m, meq = W.meq;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const double* scal = w.scal + (int64_t)kl * kScal;
  auto bail = [&]() {
    if (tid == 0) {
      b.istats[2 * k] = kNeedsGeneric;
      b.istats[2 * k + 1] = 0;
    }
  };
  if (scal[6] == 3.0) return;  // reported infeasible by the setup kernel
  if (scal[6] != 0.0 || n > RX || m > RY || n < 1) {
    bail();
    return;
  }
  // ---- LDS carve: the x-bar and y images (+ B dummy slots each for stores of non-owning lanes), the
  //      per-wave partials of the long rows / columns, reduction slots and the long-row state.
  constexpr bool PL = KR != 0;  // T(z_k) images in LDS
  double* X = reinterpret_cast<double*>(smem);
  double* Y = X + n + B;
  double* XP = Y + m + B;  // PL: x+ / y+ images of the last check, at the same byte distance D from X / Y
  double* YP = XP + n + B;
  double* TE = PL ? YP + m + B : XP;           // [WX][RX] K^T values (LDS variant)
  double* KE = TE + ((KR & 1) ? 0 : WX * RX);  // [WY][RY] K values (LDS variant)
  double* partC = KE + ((KR & 2) ? 0 : WY * RY);  // [NW][kLMax]  partial K'y of long columns
  double* partR = partC + NW * kLMax;  // [NW][kLMax]  partial K xbar of long rows
  double* red = partR + NW * kLMax;
  double* lx = red + kNRed * (NW + 1) + 4;  // long columns: x, xa, c, lo, hi, xp
  double* ly = lx + 6 * kLMax;              // long rows: y, ya, q, yp
  int32_t* ints = reinterpret_cast<int32_t*>(smem + align16(sizeof(double) * ell_lds_doubles(n, m, B, XS, YS, WX, WY, KR)));
  int32_t* lxi = ints;              // long column ids
  int32_t* lyi = ints + kLMax;      // long row ids
  int32_t* cnt = ints + 2 * kLMax;  // [0] nlx, [1] nly, [2] bad flag, [3] some wave scatters to several targets
  const int Xa = lds_addr(X), Ya = lds_addr(Y);  // absolute LDS byte addresses of the two images
  const int D = 8 * (n + m + 2 * B);              // X -> XP and Y -> YP byte distance (PL)
  const int32_t* gkp = b.indptr + W.row;
  const int32_t* gkc = b.indices + W.nz;
  const double* gkv = w.kval + W.wz;
  const int32_t* gtp = w.tptr + W.wtr;
  const int32_t* gtc = w.tind + W.wz;
  const double* gtv = w.tval + W.wz;
  const double* cs = w.cs + W.wn;
  const double* ls = w.ls + W.wn;
  const double* us = w.us + W.wn;
  const double* qs = w.qs + W.wm;
  const double* dcv = w.dc + W.wn;
  const double* drv = w.dr + W.wm;
  double* xo_g = b.x + W.on;  // x+ (scaled) at check iterations, final unscaled x
  double* yo_g = b.y + W.om;

  // ---- long lists (deterministic ballot compaction by wave 0)
  if (wid == 0) {
    int nx = 0, ny = 0;
    for (int base = 0; base < n; base += kWave) {
      const int j = base + lane;
      const bool isl = j < n && (gtp[j + 1] - gtp[j]) > WX;
      const unsigned long long bal = __ballot(isl);
      const int pre = __popcll(bal & ((1ull << lane) - 1ull));
      if (isl && nx + pre < kLMax) lxi[nx + pre] = j;
      nx += __popcll(bal);
    }
    for (int base = 0; base < m; base += kWave) {
      const int i = base + lane;
      const bool isl = i < m && (gkp[i + 1] - gkp[i]) > WY;
      const unsigned long long bal = __ballot(isl);
      const int pre = __popcll(bal & ((1ull << lane) - 1ull));
      if (isl && ny + pre < kLMax) lyi[ny + pre] = i;
      ny += __popcll(bal);
    }
    if (lane == 0) {
      cnt[0] = nx;
      cnt[1] = ny;
      cnt[2] = 0;
      cnt[3] = 0;
    }
  }
  // slot maps (in the X / Y images, as int32 before the iteration starts)
  int32_t* cmap = reinterpret_cast<int32_t*>(X);  // n ints fit in n doubles
  int32_t* rmap = reinterpret_cast<int32_t*>(Y);
  for (int j = tid; j < n; j += B) cmap[j] = -1;
  for (int i = tid; i < m; i += B) rmap[i] = -1;
  __syncthreads();
  const int nlx = cnt[0], nly = cnt[1];
  if (nlx > kLMax || nly > kLMax) {
    bail();
    return;
  }
  for (int L = tid; L < nlx; L += B) cmap[lxi[L]] = L;
  for (int L = tid; L < nly; L += B) rmap[lyi[L]] = L;
  __syncthreads();

  // ---- lane-owned state: iterate, anchor, objective, bounds, and the ELL slices of K^T (columns) and K
  //      (rows) -- values and gather offsets -- all in VGPRs for the whole solve.
  int xi[XS][WX];     // LDS byte addresses in the Y image
  constexpr bool KRX = (KR & 1) != 0, KRY = (KR & 2) != 0;
  double tk[KRX ? XS : 1][KRX ? WX : 1];  // scaled K^T values (register variant)
  int xst[XS];        // byte offset of this slot's X-image store (own column or this lane's dummy slot)
  double x[XS], xa[XS], cc[XS], lo[XS], hi[XS];
  int xs_tgt[XS];  // long K row fed by this column (scatter target)
  double xs_cf[XS];
  bool xown[XS];
#pragma unroll
  for (int s = 0; s < XS; ++s) {
    const int j = tid + s * B;
    xown[s] = false;
    xs_tgt[s] = -1;
    xs_cf[s] = 0.0;
    x[s] = xa[s] = cc[s] = lo[s] = hi[s] = 0.0;
    xst[s] = Xa + 8 * (n + tid);
    int a0 = 0, len = 0;
    if (j < n) {
      a0 = gtp[j];
      len = gtp[j + 1] - a0;
      if (len <= WX) {
        xown[s] = true;
        xst[s] = Xa + 8 * j;
        cc[s] = cs[j];
        lo[s] = ls[j];
        hi[s] = us[j];
        x[s] = xa[s] = fmin(fmax(0.0, lo[s]), hi[s]);
      }
    }
#pragma unroll
    for (int e = 0; e < WX; ++e) {
      const bool v = xown[s] && e < len;
      const int r = v ? gtc[a0 + e] : 0;
      xi[s][e] = Ya + 8 * r;
      if constexpr (KRX)
        tk[s][e] = v ? gtv[a0 + e] : 0.0;
      else
        TE[e * RX + tid + s * B] = v ? gtv[a0 + e] : 0.0;
      if (v) {
        const int L = rmap[r];
        if (L >= 0) {
          if (xs_tgt[s] >= 0) cnt[2] = 1;  // two long rows in one column: not this kernel's shape
          xs_tgt[s] = L;
          xs_cf[s] = gtv[a0 + e];
        }
      }
    }
  }
  int yi[YS][WY];     // LDS byte addresses in the X image
  double kk[KRY ? YS : 1][KRY ? WY : 1];  // scaled K values (register variant)
  int yst[YS];
  double y[YS], ya[YS], qq[YS];
  int ylo_hi[YS];  // high word of the dual lower bound: 0.0 for >= rows (i >= meq), -inf for equality rows
  int ys_tgt[YS];
  double ys_cf[YS];
  bool yown[YS];
#pragma unroll
  for (int s = 0; s < YS; ++s) {
    const int i = tid + s * B;
    yown[s] = false;
    ys_tgt[s] = -1;
    ys_cf[s] = 0.0;
    y[s] = ya[s] = qq[s] = 0.0;
    ylo_hi[s] = i >= meq ? 0 : (int)0xFFF00000;
    yst[s] = Ya + 8 * (m + tid);
    int a0 = 0, len = 0;
    if (i < m) {
      a0 = gkp[i];
      len = gkp[i + 1] - a0;
      if (len <= WY) {
        yown[s] = true;
        yst[s] = Ya + 8 * i;
        qq[s] = qs[i];
      }
    }
#pragma unroll
    for (int e = 0; e < WY; ++e) {
      const bool v = yown[s] && e < len;
      const int c = v ? gkc[a0 + e] : 0;
      yi[s][e] = Xa + 8 * c;
      if constexpr (KRY)
        kk[s][e] = v ? gkv[a0 + e] : 0.0;
      else
        KE[e * RY + tid + s * B] = v ? gkv[a0 + e] : 0.0;
      if (v) {
        const int L = cmap[c];
        if (L >= 0) {
          if (ys_tgt[s] >= 0) cnt[2] = 1;
          ys_tgt[s] = L;
          ys_cf[s] = gkv[a0 + e];
        }
      }
    }
  }
  for (int L = wid; L < nly; L += NW) {  // a long row touching a long column is not this kernel's shape
    const int i = lyi[L];
    for (int p = gkp[i] + lane; p < gkp[i + 1]; p += kWave)
      if (cmap[gkc[p]] >= 0) cnt[2] = 1;
  }
  for (int t = tid; t < 6 * kLMax; t += B) lx[t] = 0.0;
  if (tid == 0) ly[4 * kLMax] = 0.0;  // zero slot read by the long-column fast path
  __syncthreads();
  for (int L = tid; L < nlx; L += B) {
    const int j = lxi[L];
    const double l0 = ls[j], h0 = us[j], x0 = fmin(fmax(0.0, l0), h0);
    lx[L] = x0;
    lx[kLMax + L] = x0;
    lx[2 * kLMax + L] = cs[j];
    lx[3 * kLMax + L] = l0;
    lx[4 * kLMax + L] = h0;
    lx[5 * kLMax + L] = x0;
  }
  for (int L = tid; L < nly; L += B) {
    const int i = lyi[L];
    ly[L] = 0.0;
    ly[kLMax + L] = 0.0;
    ly[2 * kLMax + L] = qs[i];
    ly[3 * kLMax + L] = 0.0;
  }
  for (int t = tid; t < 2 * NW * kLMax; t += B) partC[t] = 0.0;  // partC and partR are contiguous
  // Per-wave scatter shape: when every lane of the wave feeds at most one long row (column), and all lanes
  // feed the same one, a lane sums its slots in registers and the wave needs ONE reduction per half-step.
  auto wave_target = [&](const int* tg, int S) {
    int t = -1;
    bool multi = false;
    for (int q = 0; q < S; ++q)
      if (tg[q] >= 0) {
        if (t >= 0 && t != tg[q]) multi = true;
        t = tg[q];
      }
    const unsigned long long has = __ballot(t >= 0);
    const int lead = has ? __ffsll((long long)has) - 1 : 0;
    const int tw = __shfl(t, lead, kWave);
    const bool ok = !__any(multi || (t >= 0 && t != tw));
    return has == 0ull ? -1 : (ok ? tw : -2);  // -1 none, -2 general, >= 0 the single target
  };
  const int xtw = __builtin_amdgcn_readfirstlane(wave_target(xs_tgt, XS));
  const int ytw = __builtin_amdgcn_readfirstlane(wave_target(ys_tgt, YS));
  if (lane == 0 && (xtw == -2 || ytw == -2)) cnt[3] = 1;
  if (KR && lane == 0 && (xtw == -2 || ytw == -2)) cnt[2] = 1;  // KR variants: single-target waves only
  __syncthreads();
  if (cnt[2] != 0) {
    bail();
    return;
  }
  // Partials are overwritten (single-target waves) unless some wave accumulates into several targets; then
  // every consumer must zero what it read.
  const bool zero_parts = __builtin_amdgcn_readfirstlane(cnt[3]) != 0;
  for (int i = tid; i < m; i += B) Y[i] = 0.0;
  if constexpr (PL) {  // T(z_0) = z_0 until the first check
#pragma unroll
    for (int s = 0; s < XS; ++s) lds_st(xst[s] + D, x[s]);
#pragma unroll
    for (int s = 0; s < YS; ++s) lds_st(yst[s] + D, 0.0);
    for (int L = tid; L < nlx; L += B) XP[lxi[L]] = lx[L];
    for (int L = tid; L < nly; L += B) YP[lyi[L]] = 0.0;
  }
  __syncthreads();

  double* myPC = partC + wid * kLMax;
  double* myPR = partR + wid * kLMax;
  // The dense-row contributions of this wave's slots: one DPP reduction when the wave has a single target.
  auto scatter_rows = [&](const double (&v)[XS]) {  // K xbar of long rows, from the column slots
    if (xtw >= 0) {
      double a = 0.0;
#pragma unroll
      for (int s = 0; s < XS; ++s) a += xs_cf[s] * v[s];
      a = wave_sum_dpp(a);
      if (lane == 0) myPR[xtw] = a;
    } else if (!KR && xtw == -2) {
#pragma unroll
      for (int s = 0; s < XS; ++s) wave_scatter(xs_cf[s] * v[s], xs_tgt[s], myPR);
    }
  };
  auto scatter_cols = [&](const double (&v)[YS]) {  // K'y of long columns, from the row slots
    if (ytw >= 0) {
      double a = 0.0;
#pragma unroll
      for (int s = 0; s < YS; ++s) a += ys_cf[s] * v[s];
      a = wave_sum_dpp(a);
      if (lane == 0) myPC[ytw] = a;
    } else if (!KR && ytw == -2) {
#pragma unroll
      for (int s = 0; s < YS; ++s) wave_scatter(ys_cf[s] * v[s], ys_tgt[s], myPC);
    }
  };
  auto sum_parts = [&](double* part, int L) {
    double a = 0.0;
#pragma unroll
    for (int w2 = 0; w2 < NW; ++w2) a += part[w2 * kLMax + L];
    if (zero_parts) {
#pragma unroll
      for (int w2 = 0; w2 < NW; ++w2) part[w2 * kLMax + L] = 0.0;
    }
    return a;
  };
  auto ktrans_y = [&](int s, int off = 0) {  // (K^T y)_j of column slot s from the Y image (off = D: YP)
    double a = 0.0;
#pragma unroll
    for (int e = 0; e < WX; ++e) {
      double v;
      if constexpr (KRX)
        v = tk[s][e];
      else
        v = TE[e * RX + tid + s * B];
      a = fma(v, lds_ld(xi[s][e] + off), a);
    }
    return a;
  };
  auto k_xbar = [&](int s, int off = 0) {  // (K xbar)_i of row slot s from the X image (off = D: XP)
    double a = 0.0;
#pragma unroll
    for (int e = 0; e < WY; ++e) {
      double v;
      if constexpr (KRY)
        v = kk[s][e];
      else
        v = KE[e * RY + tid + s * B];
      a = fma(v, lds_ld(yi[s][e] + off), a);
    }
    return a;
  };

  // ---- ||Kt||_2 by power iteration, v <- Kt'(Kt v) for o.power_iters steps, on chip with the same ELL
  //      slices and dense-row scatter as the half-steps; sigma^2 = |v_P| / |v_{P-1}| (no per-step
  //      normalisation: |Kt| <= 1 after Pock-Chambolle scaling, so v only shrinks by sigma^2 per step)
  double eta = scal[0];
  if (o.power_iters > 0) {
    const int P = o.power_iters;
    const double v0 = 1.0 / sqrt((double)n);
    double vc[XS];
#pragma unroll
    for (int s = 0; s < XS; ++s) vc[s] = xown[s] ? v0 : 0.0;
    double nv[2] = {0.0, 0.0};  // |v_{P-1}|^2, |v_P|^2
    for (int pi = 0; pi <= P; ++pi) {
      if (pi > 0) {  // v_pi = Kt' w (gathers of the Y image; dense columns from the row-side partials)
#pragma unroll
        for (int s = 0; s < XS; ++s) vc[s] = xown[s] ? ktrans_y(s) : 0.0;
      }
      double lv = 0.0;
      for (int L = tid; L < nlx; L += B) {
        if (pi == 0) {
          lv = v0;
        } else {
          lv = 0.0;
          for (int w2 = 0; w2 < NW; ++w2) {
            lv += partC[w2 * kLMax + L];
            partC[w2 * kLMax + L] = 0.0;
          }
        }
        X[lxi[L]] = lv;
      }
      if (pi >= P - 1) {
        double a = 0.0;
#pragma unroll
        for (int s = 0; s < XS; ++s) a += vc[s] * vc[s];
        if (tid < nlx) a += lv * lv;  // nlx <= kLMax <= B: one long column per thread at most
        nv[pi - (P - 1)] = a;
      }
      if (pi == P) break;
#pragma unroll
      for (int s = 0; s < XS; ++s)
        if (xown[s]) X[tid + s * B] = vc[s];
      scatter_rows(vc);
      __syncthreads();
      // w = Kt v (gathers of the X image; dense rows from the column-side partials)
      double wr[YS];
#pragma unroll
      for (int s = 0; s < YS; ++s) {
        wr[s] = yown[s] ? k_xbar(s) : 0.0;
        if (yown[s]) Y[tid + s * B] = wr[s];
      }
      for (int L = tid; L < nly; L += B) {
        double a = 0.0;
        for (int w2 = 0; w2 < NW; ++w2) {
          a += partR[w2 * kLMax + L];
          partR[w2 * kLMax + L] = 0.0;
        }
        Y[lyi[L]] = a;
      }
      scatter_cols(wr);
      __syncthreads();
    }
    block_sum<B, 2>(nv, red);
    if (nv[0] > 0.0 && nv[1] > 0.0) eta = o.step_safety / sqrt(sqrt(nv[1] / nv[0]));
    // back to the PDHG starting state: y = 0, empty partials
    for (int i = tid; i < m; i += B) Y[i] = 0.0;
    for (int t = tid; t < 2 * NW * kLMax; t += B) partC[t] = 0.0;
    __syncthreads();
  }
  eta = uniform(eta);
  double pw = uniform(scal[1]);
  const double cnorm = uniform(scal[2]), qnorm = uniform(scal[3]), c0 = uniform(b.c0[k]);
  int it = 0, kin = 0, status = kIterLimit;
  double r0 = -1.0, rprev = -1.0;
  double* fin = red + kNRed * NW;  // obj, pres, dres, gap of the last check (LDS, written by block_sum readers)
  if (tid == 0)
    for (int t = 0; t < 4; ++t) fin[t] = NAN;
  const int chk = o.check_every > 0 ? o.check_every : 64;

  double tau = uniform(eta / pw), sigma = uniform(eta * pw);
  const int kkt_every = o.kkt_every > 0 ? o.kkt_every : 1;
  int ck = chk, kk_ = kkt_every;
  KktGate gate;  // dvh_options.kkt_predict (as pdhg_band_kernel)
  // Halpern weights 1/(k+2): lane l holds the weight of k = kbase + l; an iteration reads its weight with
  // v_readlane (uniform lane index -> SGPRs), the slice is reloaded every 64 iterations.
  int kbase = 0;
  auto hload = [&](int k0) {
    const int kq = k0 + lane;
    return kq < kHalpernTab ? w.hinv[kq] : 1.0 / (kq + 2.0);
  };
  double hw = hload(0);

  // long-column fast path (see the primal half-step): wave 0, row r = lane / 16 <-> long column r
  const bool lc_fast = nlx <= 4 && NW <= 16 && !zero_parts;
  const bool lc_wave = lc_fast && wid == 0 && nlx > 0;
  const int lc_r = lane >> 4, lc_p = lane & 15;
  const int lc_pa = (lc_p < NW && lc_r < nlx) ? lds_addr(partC + lc_p * kLMax + lc_r) : lds_addr(ly + 4 * kLMax);
  const int lc_la = lds_addr(lx + lc_r);  // x, xa, c, lo, hi, xp at + 8 k kLMax (zeroed for r >= nlx)
  const int lc_xs = (lc_p == 0 && lc_r < nlx) ? lds_addr(X + lxi[lc_r]) : lds_addr(X + n + tid);

  // One PDHG iteration (reflected Halpern, rho = 1): z_{k+1} = ca (2 T(z_k) - z_k) + cb z_anchor.
  // CHECK iterations also accumulate the movement norms |z_k - T(z_k)|^2, |T(z_k) - z_anchor|^2 and store
  // T(z_k) for the restart / KKT checks.
  double mv0, mv1, mv2, mv3;
  auto iterate = [&](auto chk_tag, auto longc_tag) __attribute__((always_inline)) {
    constexpr bool CHECK = decltype(chk_tag)::value;
    constexpr bool LONGC = decltype(longc_tag)::value;
    if (kin - kbase >= kWave) {
      kbase = kin;
      hw = hload(kin);
    }
    const double cb = readlane_f64(hw, kin - kbase), ca = 1.0 - cb;
    mv0 = mv1 = mv2 = mv3 = 0.0;
    // ---------------- primal half-step
    {
      // Long columns (the dense DCM tau columns).  Fast path (nlx <= 4, single-target waves): wave 0 does
      // them branch-free, so it interleaves them with its own slot work: lane 16 r + p reads partial p of
      // long column r (zero slot when p >= NW or r >= nlx), a DPP row sum gives every lane of row r the
      // column's K'y (fixed order, deterministic), the row's lanes redo the same projection, and lane 16 r
      // stores it.  Otherwise one lane per long column sums the partials serially.
      double lc_kt = 0.0, lc_xo = 0.0, lc_xan = 0.0, lc_c = 0.0, lc_lo = 0.0, lc_hi = 0.0;
      if constexpr (LONGC) {
        lc_kt = row_sum16(lds_ld(lc_pa));
        lc_xo = lds_ld(lc_la);
        lc_xan = lds_ld(lc_la + 8 * kLMax);
        lc_c = lds_ld(lc_la + 16 * kLMax);
        lc_lo = lds_ld(lc_la + 24 * kLMax);
        lc_hi = lds_ld(lc_la + 32 * kLMax);
      }
      if (!lc_fast && tid < nlx) {
        const int L = tid;
        const double kt = sum_parts(partC, L);
        const int j = lxi[L];
        const double xo = lx[L], xan = lx[kLMax + L];
        const double p1 = vmin(vmax(fma(-tau, lx[2 * kLMax + L] - kt, xo), lx[3 * kLMax + L]), lx[4 * kLMax + L]);
        const double xb = fma(2.0, p1, -xo);
        X[j] = xb;
        if (CHECK) {
          const double d = xo - p1, da = p1 - xan;
          mv0 += d * d;
          mv1 += da * da;
          lx[5 * kLMax + L] = p1;
        }
        lx[L] = fma(ca, xb, cb * xan);
      }
      double kty[XS];
#pragma unroll
      for (int s = 0; s < XS; ++s) kty[s] = ktrans_y(s);
      double xbs[XS];
#pragma unroll
      for (int s = 0; s < XS; ++s) {  // branch-free: a non-owning slot has c = lo = hi = 0 and stays at 0
        const double p1 = vmin(vmax(fma(-tau, cc[s] - kty[s], x[s]), lo[s]), hi[s]);
        const double xb = fma(2.0, p1, -x[s]);
        lds_st(xst[s], xb);
        if (CHECK && xown[s]) {
          const double d = x[s] - p1, da = p1 - xa[s];
          mv0 += d * d;
          mv1 += da * da;
          if constexpr (PL)
            lds_st(xst[s] + D, p1);
          else
            xo_g[(opaque(tid) + s * B)] = p1;
        }
        x[s] = fma(ca, xb, cb * xa[s]);
        xbs[s] = xb;
      }
      if constexpr (LONGC) {
        const double p1 = vmin(vmax(fma(-tau, lc_c - lc_kt, lc_xo), lc_lo), lc_hi);
        const double xb = fma(2.0, p1, -lc_xo);
        lds_st(lc_xs, xb);  // row leaders: X[j]; other lanes: their dummy slot
        if ((lane & 15) == 0) lds_st(lc_la, fma(ca, xb, cb * lc_xan));
        if (CHECK && (lane & 15) == 0) {
          const double d = lc_xo - p1, da = p1 - lc_xan;  // zero in rows >= nlx
          mv0 += d * d;
          mv1 += da * da;
          lds_st(lc_la + 40 * kLMax, p1);
        }
      }
      scatter_rows(xbs);
    }
    lds_barrier();
    // ---------------- dual half-step
    {
      for (int L = tid; L < nly; L += B) {
        const double kv = sum_parts(partR, L);
        const int i = lyi[L];
        const double yo = ly[L], yan = ly[kLMax + L];
        double p1 = yo + sigma * (ly[2 * kLMax + L] - kv);
        if (i >= meq) p1 = fmax(p1, 0.0);
        if (CHECK) {
          const double d = yo - p1, da = p1 - yan;
          mv2 += d * d;
          mv3 += da * da;
          ly[3 * kLMax + L] = p1;
        }
        const double yn = ca * (2.0 * p1 - yo) + cb * yan;
        ly[L] = yn;
        Y[i] = yn;
      }
      double kx[YS];
#pragma unroll
      for (int s = 0; s < YS; ++s) kx[s] = k_xbar(s);
      double yns[YS];
#pragma unroll
      for (int s = 0; s < YS; ++s) {  // branch-free: a non-owning slot has q = 0 and stays at 0
        // duals of >= rows stay >= 0 (branch-free: max with 0 or -inf)
        const double p1 = vmax(fma(sigma, qq[s] - kx[s], y[s]), __hiloint2double(ylo_hi[s], 0));
        if (CHECK && yown[s]) {
          const double d = y[s] - p1, da = p1 - ya[s];
          mv2 += d * d;
          mv3 += da * da;
          if constexpr (PL)
            lds_st(yst[s] + D, p1);
          else
            yo_g[(opaque(tid) + s * B)] = p1;
        }
        const double yn = fma(ca, fma(2.0, p1, -y[s]), cb * ya[s]);
        y[s] = yn;
        lds_st(yst[s], yn);
        yns[s] = yn;
      }
      scatter_cols(yns);
    }
    ++it;
    ++kin;
    lds_barrier();
  };

  while (it < o.max_iters) {
    const bool check = --ck == 0;
    using F = std::integral_constant<bool, false>;
    using T = std::integral_constant<bool, true>;
    if (!check) {
      if (lc_wave)
        iterate(F(), T());
      else
        iterate(F(), F());
      continue;
    }
    ck = chk;
    if (lc_wave)
      iterate(T(), T());
    else
      iterate(T(), F());

    // ---------------- check (every check_every iterations): fixed-point residual of z_k, restart test;
    // every kkt_every-th check also the relative KKT error of T(z_k) = (x+, y+) in the unscaled space.
    const bool last = it + chk > o.max_iters;  // the last check before the limit is a KKT one
    bool kkt = (--kk_ == 0) || last;
    if (kkt) kk_ = kkt_every;
    double acc[kNRed];  // 0..3 movement norms, 4 ||r_p||^2, 5 ||r_d||^2, 6 c'x, 7 q'y, 8 bound term
    acc[0] = mv0;
    acc[1] = mv1;
    acc[2] = mv2;
    acc[3] = mv3;
#pragma unroll
    for (int t = 4; t < kNRed; ++t) acc[t] = 0.0;
    double r = 0.0;
    if constexpr (GATE) {  // predicted KKT gate: the restart sums first (kkt_gate_skip, dvh_device.h)
      double acc4[4] = {acc[0], acc[1], acc[2], acc[3]};
      block_sum1<B, 4, true>(acc4, red);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = acc4[t];
      r = sqrt(pw * acc[0] + acc[2] / pw);
      if (kkt && !last && kkt_gate_skip(o, gate, r)) {
        kkt = false;
        ++gate.skip;
      }
    }
    // The KKT products gather from images of T(z_k): XP / YP (PL; the long slots are copied in here), or
    // X / Y refilled from the HBM copies (restored after the check unless a restart rewrites them).
    double* const XK = PL ? XP : X;
    double* const YK = PL ? YP : Y;
    const int KO = PL ? D : 0;
    if (kkt) {
      if constexpr (!PL) {
#pragma unroll
        for (int s = 0; s < XS; ++s)
          if (xown[s]) {
            const int j = (opaque(tid) + s * B);
            X[j] = xo_g[j];
          }
#pragma unroll
        for (int s = 0; s < YS; ++s)
          if (yown[s]) {
            const int i = (opaque(tid) + s * B);
            Y[i] = yo_g[i];
          }
      }
      for (int L = tid; L < nlx; L += B) XK[lxi[L]] = lx[5 * kLMax + L];
      for (int L = tid; L < nly; L += B) YK[lyi[L]] = ly[3 * kLMax + L];
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
        if (DVH_KKT_RDX) acc[kRdx] += fabs(rd) * fabs(xj * d);
      };
      auto row_kkt = [&](int i, double kv, double qi, double yi2) {
        const double d = drv[opaque(i)];
        double r = (qi - kv) / d;
        if (i >= meq) r = fmax(r, 0.0);
        acc[4] += r * r;
        acc[7] += qi * yi2;
        acc[9] += (yi2 * d) * (yi2 * d);
      };
#pragma unroll
      for (int s = 0; s < XS; ++s)
        if (xown[s]) col_kkt(tid + s * B, ktrans_y(s, KO), cc[s], lo[s], hi[s], XK[tid + s * B]);
#pragma unroll
      for (int s = 0; s < YS; ++s)
        if (yown[s]) row_kkt(tid + s * B, k_xbar(s, KO), qq[s], YK[tid + s * B]);
      // long rows / columns: wave gathers from the workspace CSR (termination checks only)
      for (int L = wid; L < nlx; L += NW) {
        const int j = lxi[L];
        double kt = 0.0;
        for (int p = gtp[j] + lane; p < gtp[j + 1]; p += kWave) kt += gtv[p] * YK[gtc[p]];
        kt = wave_sum_dpp(kt);
        if (lane == 0) col_kkt(j, kt, lx[2 * kLMax + L], lx[3 * kLMax + L], lx[4 * kLMax + L], lx[5 * kLMax + L]);
      }
      for (int L = wid; L < nly; L += NW) {
        const int i = lyi[L];
        double kv = 0.0;
        for (int p = gkp[i] + lane; p < gkp[i + 1]; p += kWave) kv += gkv[p] * XK[gkc[p]];
        kv = wave_sum_dpp(kv);
        if (lane == 0) row_kkt(i, kv, ly[2 * kLMax + L], ly[3 * kLMax + L]);
      }
    }
    // readlane broadcast: the sums (and all decisions below) are uniform.  A restart-only check needs the
    // four movement norms alone (each wave-wide sum is ~25 VALU ops).
    if constexpr (GATE) {
      if (kkt) {  // the KKT sums in the slots after the restart sums'
        double acc6[kNRed - 4];
#pragma unroll
        for (int t = 4; t < kNRed; ++t) acc6[t - 4] = acc[t];
        block_sum1<B, kNRed - 4, true>(acc6, red + 4 * NW);
#pragma unroll
        for (int t = 4; t < kNRed; ++t) acc[t] = acc6[t - 4];
      }
    } else if (kkt) {
      block_sum1<B, kNRed, true>(acc, red);
    } else {
      double acc4[4] = {acc[0], acc[1], acc[2], acc[3]};
      block_sum1<B, 4, true>(acc4, red);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = acc4[t];
    }
    if constexpr (!GATE) r = sqrt(pw * acc[0] + acc[2] / pw);
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
      if (kkt_done(o, pres, dres, gap, pobj, dobj, acc[4], acc[9], DVH_KKT_RDX ? acc[kRdx] : 0.0)) {
        status = kOptimal;
        break;
      }
      if constexpr (GATE) gate.note(pres, dres, gap, o.eps, r);
      if (!(isfinite(pobj) && isfinite(dobj))) {
        status = kNumerical;
        break;
      }
    }
    if (r0 < 0.0) r0 = r;
    const bool restart = (r <= o.b_suff * r0) || (r <= o.b_nec * r0 && rprev >= 0.0 && r > rprev) ||
                         ((double)kin >= o.b_art * (double)it);
    if (restart) {
      const double ddx = sqrt(acc[1]), ddy = sqrt(acc[3]);
      if (ddx > 1e-10 && ddy > 1e-10) pw = uniform(pw_update(ddy / ddx, pw, o.theta));
      tau = uniform(eta / pw);
      sigma = uniform(eta * pw);
      double yns[YS];
#pragma unroll
      for (int s = 0; s < XS; ++s)
        if (xown[s]) x[s] = xa[s] = PL ? lds_ld(xst[s] + D) : xo_g[(opaque(tid) + s * B)];
#pragma unroll
      for (int s = 0; s < YS; ++s) {
        yns[s] = 0.0;
        if (yown[s]) {
          const int i = (opaque(tid) + s * B);
          y[s] = ya[s] = yns[s] = PL ? lds_ld(yst[s] + D) : yo_g[i];
          Y[i] = y[s];
        }
      }
      for (int L = tid; L < nlx; L += B) lx[L] = lx[kLMax + L] = lx[5 * kLMax + L];
      for (int L = tid; L < nly; L += B) {
        ly[L] = ly[kLMax + L] = ly[3 * kLMax + L];
        Y[lyi[L]] = ly[L];
      }
      // the long columns' K'y partials must now refer to y = y+: rebuild this wave's row
      if (lane < kLMax) myPC[lane] = 0.0;
      scatter_cols(yns);
      kin = 0;
      kbase = 0;
      hw = hload(0);
      r0 = r;
      rprev = -1.0;
    } else {
      rprev = r;
      if (kkt && !PL) {
#pragma unroll
        for (int s = 0; s < YS; ++s)
          if (yown[s]) Y[tid + s * B] = y[s];
        for (int L = tid; L < nly; L += B) Y[lyi[L]] = ly[L];
      }
    }
    lds_barrier();
  }
  // outputs: the last check's T(z_k), unscaled
#pragma unroll
  for (int s = 0; s < XS; ++s)
    if (xown[s]) xo_g[tid + s * B] = (PL ? lds_ld(xst[s] + D) : xo_g[tid + s * B]) * dcv[tid + s * B];
  for (int L = tid; L < nlx; L += B) xo_g[lxi[L]] = lx[5 * kLMax + L] * dcv[lxi[L]];
#pragma unroll
  for (int s = 0; s < YS; ++s)
    if (yown[s]) yo_g[tid + s * B] = (PL ? lds_ld(yst[s] + D) : yo_g[tid + s * B]) * drv[tid + s * B];
  for (int L = tid; L < nly; L += B) yo_g[lyi[L]] = ly[3 * kLMax + L] * drv[lyi[L]];
  if (tid == 0) {
    b.istats[2 * k] = status;
    b.istats[2 * k + 1] = it;
    for (int t = 0; t < 4; ++t) b.stats[4 * k + t] = fin[t];
  }
}

template <int B, int XS, int YS, bool MLDS>
hipError_t launch_one(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, size_t lds, hipStream_t s,
                      const int32_t* list, int nlist) {
  auto kern = pdhg_kernel<B, XS, YS, MLDS>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(list ? nlist : ch.count), dim3(B), lds, s, b, w, ch, o, list);
  return hipGetLastError();
}

// 512-thread workgroups (8 waves, up to 256 VGPRs per lane): each lane owns up to 8 columns and 8 rows,
// so windows with n, m <= 4096 run with the whole iterate in registers.
template <bool MLDS>
hipError_t dispatch_xy(int xs, int ys, const Batch& b, const Work& w, const Chunk& ch, const Opts& o, size_t lds,
                       hipStream_t s, const int32_t* list, int nlist) {
  constexpr int B = 512;
#define DVH_CASE(X_, Y_) \
  if (xs <= X_ && ys <= Y_) return launch_one<B, X_, Y_, MLDS>(b, w, ch, o, lds, s, list, nlist);
  DVH_CASE(2, 2)
  DVH_CASE(5, 3)
  DVH_CASE(6, 4)
  DVH_CASE(6, 6)
  DVH_CASE(8, 8)
#undef DVH_CASE
  return hipErrorInvalidValue;
}

template <int B, int XS, int YS, int WX, int WY, int KR, int WPE = 1>
hipError_t launch_ell_one(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n, int max_m,
                          hipStream_t s, const int32_t* list, int nlist) {
  const size_t lds = ell_lds_bytes(max_n, max_m, B, XS, YS, WX, WY, KR);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  auto kern = o.kkt_predict > 0 ? pdhg_ell_kernel<B, XS, YS, WX, WY, KR, WPE, true>
                                : pdhg_ell_kernel<B, XS, YS, WX, WY, KR, WPE, false>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(list ? nlist : ch.count), dim3(B), lds, s, b, w, ch, o, list);
  return hipGetLastError();
}

// Instantiations, tried in order; the first whose slots cover (n, m) and whose LDS fits is launched.
// KR variants keep K / K^T in VGPRs: 768-thread workgroups (12 waves, <= 168 VGPRs) cover the monthly
// battery + DCM window (n <= 2304, m <= 1536) with three waves per SIMD; larger windows keep the values in
// LDS with 512 threads.
#ifndef DVH_KR768
#define DVH_KR768 -1
#endif
// K and K^T in VGPRs for the narrow <2,4> slices (the monthly battery + DCM window: measured 1.40 vs 1.59
// us per window-iteration per CU against K^T in LDS).
template <int WX, int WY>
constexpr int kr768() { return DVH_KR768 >= 0 ? DVH_KR768 : 3; }
template <int WX, int WY>
hipError_t ell_dispatch_xy(int max_n, int max_m, const Batch& b, const Work& w, const Chunk& ch, const Opts& o,
                           hipStream_t s, int* variant_out, const int32_t* list, int nlist) {
  // (instantiations whose ELL slices alone exceed the LDS are never launchable and are not compiled: <512,5,3> of the
  // <4,8> slices; the <512,6,4> / <512,8,6> ones of both, which had spilled 78-698 VGPRs, are gone)
#define DVH_CASE(B_, X_, Y_, KR_)                                                                                 \
  if constexpr (ell_lds_bytes(0, 0, B_, X_, Y_, WX, WY, KR_) <= 160 * 1024) {                                     \
    if (max_n <= X_ * B_ && max_m <= Y_ * B_ && ell_lds_bytes(max_n, max_m, B_, X_, Y_, WX, WY, KR_) <= 160 * 1024) { \
      if (variant_out)                                                                                            \
        *variant_out = (2000000 + 1000000 * KR_) + WX * 100000 + WY * 10000 + (B_ / 64) * 100 + X_ * 10 + Y_;     \
      return launch_ell_one<B_, X_, Y_, WX, WY, KR_>(b, w, ch, o, max_n, max_m, s, list, nlist);                  \
    }                                                                                                             \
  }
  DVH_CASE(512, 1, 1, 3)
  DVH_CASE(512, 2, 2, 3)
#ifndef DVH_NO768
  // <2,4> slices only: the <4,8> form (K in VGPRs) spilled 144-165 VGPRs at the 768-thread budget, and no measured
  // workload reached it (POI windows of 1,921 columns refuse the ELL shape, profiles/r05y_poi_paths.log)
  if constexpr (WX <= 2 && WY <= 4) {
    DVH_CASE(768, 3, 2, (kr768<WX, WY>()))
  }
#endif
  DVH_CASE(512, 5, 3, 0)
  // (<512,6,4> of the <2,4> slices dropped: 61-72 spilled VGPRs and no measured workload -- its windows, n in
  // (2560, 3072], take the generic kernel)
#undef DVH_CASE
  return hipErrorInvalidValue;
}

}  // namespace

int setup_segments(int max_n) { return max_n <= 8000 ? 4 : 1; }
size_t setup_lds_bytes(int max_n, int max_m) {
  // transpose cursors, later reused for Dr / Dc
  return align16(std::max(sizeof(int32_t) * (size_t)setup_segments(max_n) * ((size_t)max_n + 1),
                          sizeof(double) * ((size_t)max_n + (size_t)max_m)));
}

hipError_t launch_setup(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n, int max_m,
                        hipStream_t s, const int32_t* list, int nlist) {
  const size_t lds = setup_lds_bytes(max_n, max_m);
  Opts o2 = o;
  o2.setup_segments = setup_segments(max_n);
  hipError_t e = hipFuncSetAttribute((const void*)setup_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  const int nb = list ? nlist : ch.count;
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(setup_kernel<false>, dim3(nb), dim3(kSetupB), lds, s, b, w, ch, o2, list);
  return hipGetLastError();
}

hipError_t launch_setup_medium(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n,
                               const int32_t* list, int nlist, hipStream_t s) {
  Opts o2 = o;
  o2.setup_segments = setup_segments(max_n);
  const size_t lds = align16(sizeof(int32_t) * (size_t)o2.setup_segments * ((size_t)max_n + 1));
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)setup_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(setup_kernel<true>, dim3(nlist), dim3(kSetupB), lds, s, b, w, ch, o2, list);
  return hipGetLastError();
}

hipError_t launch_power(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, const int32_t* list, int nlist,
                        hipStream_t s) {
  hipLaunchKernelGGL(power_kernel, dim3(nlist), dim3(kSetupB), 0, s, b, w, ch, o, list);
  return hipGetLastError();
}

hipError_t launch_pdhg(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n, int max_m,
                       int64_t max_nnz, hipStream_t s, int* variant_out, const int32_t* list, int nlist) {
  constexpr int B = 512;
  constexpr size_t kLdsCap = 160 * 1024;
  const int xs = (max_n + B - 1) / B, ys = (max_m + B - 1) / B;
  if (xs > 8 || ys > 8) return hipErrorInvalidValue;
  const size_t lds_m = pdhg_lds_bytes(max_n, max_m, (int)max_nnz, true, B / kWave);
  const bool mlds = lds_m <= kLdsCap && max_n < 65536 && max_m < 65536;
  const size_t lds = mlds ? lds_m : pdhg_lds_bytes(max_n, max_m, 0, false, B / kWave);
  if (lds > kLdsCap) return hipErrorInvalidValue;
  if (variant_out) *variant_out = (mlds ? 1000 : 0) + xs * 10 + ys;
  return mlds ? dispatch_xy<true>(xs, ys, b, w, ch, o, lds, s, list, nlist)
              : dispatch_xy<false>(xs, ys, b, w, ch, o, lds, s, list, nlist);
}

// Small windows (the daily market-service window: T = 24, n = 168, m <= 265, K^T rows <= 6, K rows <= 8; with
// SR + NSR n = 264, with load following n = 408, m <= 505): one four-wave workgroup per window with K and K^T values
// in VGPRs (one column and two rows per lane up to n = 256, two and two up to 512) -- spill-free, two windows per CU.
// 1,095 Usecase 3 days (MARKET_OPTIONS): 5.3 ms (DA + FR), 5.7 ms (+ SR + NSR), 9.9 ms (+ LF), 15.5 ms (CombinedMarket
// LF), against 11.3 / 17.4 / 11.2 / 47.7 ms for the round-4 table of one- and two-wave variants, whose register
// budgets spilled 19-245 VGPRs (profiles/r05w_market_variants.log, r05x_market_candidates*.log).
static int small_variant() {  // DVH_SMALL=-1: off (A/B against the 512-thread kernels); 0..2: force a variant
  static const int v = getenv("DVH_SMALL") ? atoi(getenv("DVH_SMALL")) : 99;
  return v;
}
// DVH_SMALL_LATENCY=0/1: skip all / take all small variants for batches of at most two windows per CU (A/B)
static int small_latency() {
  static const int v = getenv("DVH_SMALL_LATENCY") ? atoi(getenv("DVH_SMALL_LATENCY")) : -1;
  return v;
}

hipError_t small_dispatch(int max_n, int max_m, int wx, int wy, const Batch& b, const Work& w, const Chunk& ch,
                          const Opts& o, hipStream_t s, int* variant_out, const int32_t* list, int nlist,
                          bool latency) {
  const int sv = small_variant();
#define DVH_SMALL(V_, B_, X_, Y_, WX_, WY_, KR_, WPE_)                                                          \
  if ((sv == 99 || sv == V_) && max_n <= X_ * B_ && max_m <= Y_ * B_ && wx <= WX_ && wy <= WY_) {             \
    if (variant_out)                                                                                          \
      *variant_out = (2000000 + 1000000 * KR_) + WX_ * 100000 + WY_ * 10000 + (B_ / 64) * 100 + X_ * 10 + Y_; \
    return launch_ell_one<B_, X_, Y_, WX_, WY_, KR_, WPE_>(b, w, ch, o, max_n, max_m, s, list, nlist);       \
  }
  DVH_SMALL(0, 256, 1, 2, 6, 8, 3, 1)
  // two columns per lane: behind the 512-thread ELL kernel for batches of at most two windows per CU (load-following
  // days, n = 408: 7.6 vs 6.5 ms for 366 windows), ahead of it beyond (9.98 vs 11.3 ms for 1,095); ahead of the
  // generic kernel, which takes K^T rows wider than 4, at every size (SR + NSR days: 1.9 vs 3.9 ms for 15 windows)
  if (latency && small_latency() != 1 && wx <= 4) return hipErrorInvalidValue;
  DVH_SMALL(1, 256, 2, 2, 6, 8, 3, 1)
  // m up to 768 with K^T rows of 5-6 entries (beyond the 512-thread kernels' width 4): K and K^T values in LDS.
  // Windows the 512-thread kernels take (K^T width <= 4, m just above 512) run 2.9x faster there
  // (profiles/r02zj_market_variants.log)
  if (wx > 4 || sv == 2) {
    DVH_SMALL(2, 256, 2, 3, 6, 8, 0, 2)
  }
#undef DVH_SMALL
  return hipErrorInvalidValue;
}
static bool small_enabled() { return small_variant() >= 0; }

hipError_t launch_pdhg_ell(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n, int max_m,
                           int wx, int wy, hipStream_t s, int* variant_out, const int32_t* list, int nlist,
                           bool latency) {
  // latency: few windows (at most two per CU) -- the small variants that beat the 512-thread kernels there (DA + FR
  // days: 1.7 vs 3.8 ms for 15 windows, 3.7 vs 8.8 ms for 366 against the generic kernel,
  // profiles/r05y_market_table.log; DVH_SMALL_LATENCY=0 skips them, =1 takes all)
  if (max_n <= 512 && max_m <= 768 && wx <= 6 && wy <= 8 && small_enabled() && (!latency || small_latency() != 0)) {
    const hipError_t e = small_dispatch(max_n, max_m, wx, wy, b, w, ch, o, s, variant_out, list, nlist, latency);
    if (e != hipErrorInvalidValue) return e;
    (void)hipGetLastError();  // no small variant covers the shape (e.g. DVH_SMALL forcing one): the 512-thread kernels
  }
  if (wx <= 2 && wy <= 4) return ell_dispatch_xy<2, 4>(max_n, max_m, b, w, ch, o, s, variant_out, list, nlist);
  if (wx <= 4 && wy <= 8) return ell_dispatch_xy<4, 8>(max_n, max_m, b, w, ch, o, s, variant_out, list, nlist);
  return hipErrorInvalidValue;
}

}  // namespace dvh

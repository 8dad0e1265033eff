// dvh_chain.hip -- the medium tier: battery windows longer than one workgroup (T > 768 steps, e.g. the annual
// hourly window n = "year", T = 8,760, or a 15-minute monthly window, T = 2,976; Model_Parameters_Template_DER.csv
// `n`, `dt`), solved as a batch.
//
// A window is cut into P <= kPMax segments of <= 768 consecutive time steps; each segment is one 768-thread
// workgroup that runs the battery-banded PDHG of dvh_band.hip on its steps (lane = step, every coefficient and
// iterate in VGPRs), and the P workgroups of a window form a team that advances in lock step.  What couples the
// segments each iteration (teams are formed from workgroups that share an XCD where the grid allows: one L2 for
// the hand-offs; windows are handed out dynamically, one atomic per window, so a slow window does not idle the
// rest of the chip):
//   * the SOE chain: the SOE row of the last step of segment s-1 (the boundary row) couples that step's ch, dis,
//     ene with the first ene of segment s.  Segment s-1 owns the row; segment s keeps a ghost copy (wave 0, the
//     last lane) and repeats its dual update with the same operands in the same order, so the copies are
//     bit-identical and s never needs the row's dual from s-1.  After each primal half-step, s-1 sends the
//     reflected ch, dis, ene of its last step up and s sends the reflected first ene down: ONE exchange per
//     iteration, both directions at once;
//   * DCM demand columns (tau) whose rows lie in several segments: every segment holding rows of a tau column
//     publishes its partial K'y sum for it at the start of the primal half-step and collects the others' after
//     its own primal work (the column's x-bar is needed only in the dual half-step, so this hop overlaps the
//     other); every such segment performs the column's update redundantly from the partials summed in segment
//     order, so all copies are bit-identical.  The plan cuts segments at demand-period boundaries where it can
//     (the annual window's months are segments of their own), so most windows share no column;
//   * the restart / termination checks (every check_every iterations): per-segment partial sums, added in segment
//     order by every segment, so every segment takes the same decision.
// The hand-offs are 8-byte {tag, 32-bit half} granules written by one relaxed agent-scope atomic store and polled
// by relaxed agent-scope loads (MI355X_MICROARCH.md, inter-workgroup visibility: granules need no fence); tags are
// (window ordinal, round), so no flag or buffer ever needs resetting inside a launch, and every buffer is
// double-buffered by round parity (a producer can be at most one round ahead of any consumer, because it needs the
// consumer's data of the round in between).  Teams are persistent: one launch of the device's resident capacity of
// workgroups, team t taking windows t, t + NT, ...; every spin is bounded and an expired one aborts the launch (the
// host hands the unfinished windows to the grid-wide path), so a fault can never leave waves spinning.
//
// Same algorithm, scaling, steps and checks as the band kernel (restated in oracle/pdlp_ref.py); a segment's
// arithmetic is the band kernel's for its steps, so results agree with the on-chip kernels to rounding.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "dvh_device.h"

namespace dvh {
namespace {

constexpr int kCB = kChainB;  // threads (and maximum steps) per segment
#ifndef DVH_CHAIN_TAU_WAVE
#define DVH_CHAIN_TAU_WAVE 1
#endif
constexpr int kTauWave = DVH_CHAIN_TAU_WAVE;  // the wave holding the tau slots (wave 0 holds the init / ghost row)
// DVH_CHAIN_PRIO (round 6, A/B, off): s_setprio for the waves whose primal half-step ends in a hand-off (as the band
// kernel's wave 0, DVH_BAND_PRIO), until they have published.  DVH_CHAIN_KKT_PREFETCH (A/B, off): a KKT check's factor
// loads issued together at the top of the check (as the band kernel's).  Measured and not kept
// (profiles/r06f_chain_ab.log): config 3 DCM + PV 6.6 / 6.6 windows/s with prefetch / + priority against 6.8 without
// (the prefetched doubles raise the spills 25 -> 36 VGPRs around the out-of-line KKT helpers), medium annual 1,526 /
// 1,522 against 1,610: the team kernel runs one segment per CU, so there is no other workgroup to take issue slots from.
#ifndef DVH_CHAIN_PRIO
#define DVH_CHAIN_PRIO 0
#endif
#ifndef DVH_CHAIN_KKT_PREFETCH
#define DVH_CHAIN_KKT_PREFETCH 0
#endif
static_assert(kTauWave >= 0 && kTauWave < kCB / kWave, "the tau wave exists");
constexpr int kJSeg = kChainJSeg;  // tau columns per segment
// granule offsets inside a segment's area (p = round parity)
constexpr int kCW = 2 * kNRed;  // granules per parity of the check sums (two per value)
constexpr int kOffD = 0;      // + 2p: reflected first ene (down, to s-1)
constexpr int kOffU = 4;      // + 6p: reflected ch, dis, ene of the last step (up, to s+1)
constexpr int kOffA2 = 16;    // + 8p + 2u: partial K'y of tau slot u
constexpr int kOffK = 32;     // + 12p: KKT images {first ene, 4 tau partials}
constexpr int kOffC = 56;     // + kCW p + 2v: check partial sums
constexpr int kOffW = kOffC + 2 * kCW;  // + p: the team's next window (segment 0's area)
constexpr int kOffAck = kOffW + 2;      // + p: this segment has read it
constexpr int kOffT = kOffAck + 2;      // + kCW p + 2v: check sums over all segments (segment 0's area: the leader's)
constexpr int kXSeg = kOffT + 2 * kCW;  // granules per segment in the exchange buffer
// poll-list entries per segment: A [0, 256), K [256, 512), C [512, 1016), up [1016, 1022), down [1022, 1024)
constexpr int kPollMax = 1024;
constexpr int kPollK = 256, kPollC = 512, kPollU = 1016, kPollD = 1022;
static_assert(kPMax - 1 <= kPollU - kPollC, "the window hand-out's acknowledgements fit the C list");

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gi32;

// KKT pieces of one column / one row, out of line (DVH_CHAIN_KKT_INLINE 0, the default): the check runs every
// kkt_every * check_every iterations.  Inlined they were 1 % faster while this unit was built with machine LICM; built
// without it (build.py), out of line is faster: config 3 DCM + PV 148 -> 146 ms, medium annual 646 -> 618 ms
// (profiles/r05zz_chain_kkt_outofline.log)
struct ColKktC {
  double rd2, cx, bt, rdx;
};
#ifndef DVH_CHAIN_KKT_INLINE
#define DVH_CHAIN_KKT_INLINE 0
#endif
#if DVH_CHAIN_KKT_INLINE
#define DVH_CHAIN_KKT_FN __forceinline__
#else
#define DVH_CHAIN_KKT_FN __noinline__
#endif
__device__ DVH_CHAIN_KKT_FN ColKktC col_kkt_c(double kt, double cj, double loj, double hij, double xj, double d) {
  const double rc = (cj - kt) / d;
  const bool fl = isfinite(loj), fh = isfinite(hij);
  const double lam = (fl && fh) ? rc : (fl ? fmax(rc, 0.0) : (fh ? fmin(rc, 0.0) : 0.0));
  const double rd = rc - lam;
  return {rd * rd, cj * xj, (fl ? loj * d * fmax(lam, 0.0) : 0.0) + (fh ? hij * d * fmin(lam, 0.0) : 0.0),
          fabs(rd) * fabs(xj * d)};
}
struct RowKktC {
  double rp2, y2;
};
__device__ DVH_CHAIN_KKT_FN RowKktC row_kkt_c(double kv, double qi, double yi, double dr, bool ge) {
  double r = (qi - kv) / dr;
  if (ge) r = fmax(r, 0.0);
  return {r * r, (yi * dr) * (yi * dr)};
}

__device__ __forceinline__ unsigned chain_tag(int wseq, int round) {
  return ((unsigned)(wseq & 0x3FFF) << 18) | ((unsigned)round & 0x3FFFFu);
}
// one double as two granules {tag, hi} {tag, lo}
__device__ __forceinline__ void put_f64(gu64* g, unsigned tag, double v) {
  const unsigned long long t = (unsigned long long)tag << 32;
  __hip_atomic_store(g, t | (unsigned)__double2hiint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, t | (unsigned)__double2loint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS layout (doubles): XE[B+1] YS[B+1] XT[4] XK[4] GK[4] red[kNRed(NW+1)+4] TP[4][B] XP[3][B] YP[2][B]
//   CR[kPMax][kNRed]
//   RO[6][B] (objective and upper bound of the lane's ch, dis, ene: read-only, kept out of VGPRs)
//   | ints: poll offsets [kPollMax], poll values [kPollMax], misc[32]
__host__ __device__ inline size_t chain_lds_doubles() {
  const int NW = kCB / kWave;
  return 2 * (size_t)(kCB + 1) + 12 + (size_t)kNRed * (NW + 1) + 4 + (size_t)kJSeg * kCB + 5 * (size_t)kCB +
         (size_t)kPMax * kNRed + 6 * (size_t)kCB;
}
__host__ __device__ inline size_t chain_lds_bytes() {
  return align16(sizeof(double) * chain_lds_doubles()) + sizeof(int32_t) * (2 * (size_t)kPollMax + 32);
}

// ---------------------------------------------------------------------------------------------------------------
// Plan: one workgroup per listed window, before the setup (it reads only the window's unscaled data).  Reports crossed
// bounds (plan[0] = -1, status PRIMAL_INFEASIBLE as the setup kernel would), verifies the battery + DCM pattern (as
// the band kernel), writes the step -> DCM row / tau maps into the window's vbuf workspace, and cuts the steps into
// segments greedily: a new segment starts when the current one holds kCB steps, when a step brings a tau column the
// segment has no slot left for, or where a run of steps of one tau column begins that would not end inside the
// current segment but fits in a segment of its own (so demand periods that fit are not split).  The greedy walks the
// RUNS of equal tau ids (compacted in parallel), not the steps: a 5-minute annual window (105,120 steps) with monthly
// demand columns has 12 runs.  A column's sharers must be a contiguous range of segments; a segment inside the range
// that has none of the column's rows holds it in a free slot (its partials are zero), or the window is not planned.
// plan[0] = P (0: not this tier, -1: crossed bounds, reported).
// ---------------------------------------------------------------------------------------------------------------
constexpr int kPlanB = 1024;
constexpr int kRunsLds = 16384;  // run starts staged in LDS; more runs are read from the window's wbuf workspace

__global__ __launch_bounds__(kPlanB) void chain_plan_kernel(const Batch b, const Work w, const Chunk ch,
                                                            const int32_t* list, int32_t* plan) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int32_t* rs_lds = reinterpret_cast<int32_t*>(smem);  // [kRunsLds + 1] run starts
  __shared__ int32_t colLo[kChainJMax], colHi[kChainJMax];
  __shared__ int32_t set[kJSeg];
  __shared__ int32_t wtot[kPlanB / kWave];
  const int k = list[blockIdx.x];
  const WinOff W = win_offsets(b, ch, k);
  const int n = W.n, m = W.m, meq = W.meq;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int32_t* pl = plan + (int64_t)blockIdx.x * kPlanInts;
  // 0. crossed bounds: infeasible as given (as setup_kernel step 0)
  {
    int crossed = 0;
    for (int j = tid; j < n; j += kPlanB) crossed |= b.l[W.on + j] > b.u[W.on + j];
    if (__syncthreads_or(crossed)) {
      if (tid == 0) {
        pl[0] = -1;
        w.scal[(int64_t)(k - ch.first) * kScal + 6] = 3.0;
        b.istats[2 * k] = 1;  // DVH_PRIMAL_INFEASIBLE
        b.istats[2 * k + 1] = 0;
        for (int u = 0; u < 4; ++u) b.stats[4 * k + u] = u == 0 ? NAN : 0.0;
      }
      return;
    }
  }
  const int T = meq - 1, J = n - 3 * T, MI = m - meq;
  if (T < 1 || T > kPMax * kCB || J < 0 || J > kChainJMax || MI < 0 || MI > T || (J == 0 && MI > 0)) {
    if (tid == 0) pl[0] = 0;
    return;
  }
  const int32_t* gkp = b.indptr + W.row;
  const int32_t* gkc = b.indices + W.nz;
  const double* lo = b.l + W.on;
  int32_t* dm = reinterpret_cast<int32_t*>(w.vbuf + W.wn);  // [T] DCM row, [T..2T) tau id
  for (int t = tid; t < T; t += kPlanB) {
    dm[t] = -1;
    dm[T + t] = -1;
  }
  for (int j = tid; j < kChainJMax; j += kPlanB) {
    colLo[j] = 0x7fffffff;
    colHi[j] = -1;
  }
  __syncthreads();
  int bad = 0;
  for (int r = tid; r <= T; r += kPlanB) {
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
    bad |= lo[t] != 0.0 || lo[T + t] != 0.0;  // no lower bound kept for ch / dis (l / Dc == 0 iff l == 0)
  }
  for (int i = meq + tid; i < m; i += kPlanB) {
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
    if (atomicCAS(&dm[tc], -1, i) != -1) {  // at most one DCM row per step
      bad = 1;
      continue;
    }
    dm[T + tc] = jj;
  }
  if (__syncthreads_or(bad)) {
    if (tid == 0) pl[0] = 0;
    return;
  }
  // 1. runs of equal tau ids: starts compacted in step order (ballot per wave, wave totals scanned per chunk)
  int32_t* rs_g = reinterpret_cast<int32_t*>(w.wbuf + W.wm);  // [T + 1] when they do not fit LDS (m >= T + 1)
  int R = 0;
  for (int base = 0; base < T; base += kPlanB) {
    const int t = base + tid;
    const bool st = t < T && (t == 0 || dm[T + t] != dm[T + t - 1]);
    const unsigned long long bal = __ballot(st);
    if (lane == 0) wtot[wid] = __popcll(bal);
    __syncthreads();
    int off = R;
    for (int u = 0; u < wid; ++u) off += wtot[u];
    int tot = 0;
    for (int u = 0; u < kPlanB / kWave; ++u) tot += wtot[u];
    if (st) {
      const int pos = off + __popcll(bal & ((1ull << lane) - 1ull));
      rs_g[pos] = t;
      if (pos < kRunsLds) rs_lds[pos] = t;
    }
    R += tot;
    __syncthreads();
  }
  __syncthreads();
  // 2. the greedy over the runs (thread 0)
  if (tid == 0) {
    const int32_t* rs = R < kRunsLds ? rs_lds : rs_g;
    const int32_t* jl = dm + T;
    int P = 0, s0 = 0, ns = 0, ok = 1;
    pl[kPlanStart] = 0;
    auto close = [&](int t) {  // segment P = [s0, t)
      if (P >= kPMax) {
        ok = 0;
        return;
      }
      for (int u = 0; u < kJSeg; ++u) {
        const int id = u < ns ? set[u] : -1;
        pl[kPlanSlot + 4 * P + u] = id;
        if (id >= 0) {
          colLo[id] = min(colLo[id], P);
          colHi[id] = max(colHi[id], P);
        }
      }
      ++P;
      pl[kPlanStart + P] = t;
      s0 = t;
      ns = 0;
    };
    for (int r = 0; r < R && ok; ++r) {
      const int a = rs[r], e = r + 1 < R ? rs[r + 1] : T;
      const int j = jl[a];
      bool newj = j >= 0;
      for (int u = 0; u < ns && newj; ++u) newj = set[u] != j;
      const bool run_cut = a > s0 && e - s0 > kCB && e - a <= kCB;
      if (a - s0 == kCB || (newj && ns == kJSeg) || run_cut) {
        close(a);
        newj = j >= 0;
      }
      if (newj && ok) set[ns++] = j;
      while (ok && e - s0 > kCB) {  // full segments inside the run
        close(s0 + kCB);
        if (j >= 0) set[ns++] = j;
      }
    }
    if (ok) close(T);
    // sharers: a contiguous range of segments, each holding the column in a slot (a free slot if it has no rows)
    for (int jj = 0; jj < J && ok; ++jj) {
      if (colHi[jj] < 0) {
        ok = 0;  // a tau column without rows: its update has no owner
        break;
      }
      for (int sg = colLo[jj] + 1; sg < colHi[jj] && ok; ++sg) {
        int u = 0, fr = -1;
        for (; u < kJSeg; ++u) {
          const int id = pl[kPlanSlot + 4 * sg + u];
          if (id == jj) break;
          if (id < 0 && fr < 0) fr = u;
        }
        if (u == kJSeg) {
          if (fr < 0) ok = 0;
          else pl[kPlanSlot + 4 * sg + fr] = jj;
        }
      }
    }
    for (int sg = 0; sg < P && ok; ++sg)
      for (int u = 0; u < kJSeg; ++u) {
        const int id = pl[kPlanSlot + 4 * sg + u];
        pl[kPlanLo + 4 * sg + u] = id >= 0 ? colLo[id] : 0;
        pl[kPlanHi + 4 * sg + u] = id >= 0 ? colHi[id] : -1;
      }
    pl[1] = T;
    pl[2] = J;
    pl[3] = k;
    pl[0] = ok ? P : 0;
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Grid-wide setup of one planned window too large for the one-workgroup setup kernel (n >= kMedSetupNMax: the
// 5-minute annual window).  The same scaling as setup_kernel (Ruiz inf-norm passes, one Pock-Chambolle pass,
// oracle/pdlp_ref.py), with the columns' entries located through the plan's step maps instead of a transpose: ch_t
// and dis_t sit in row t + 1 (their SOE row) and their DCM row, ene_t in rows t and t + 1, tau_j in the DCM rows of
// its steps (a workgroup per tau column, fixed summation order).  Writes what the chain kernel reads: scaled K in CSR
// order (kval), Dr / Dc, scaled c / l / u / q, and scal[0..3, 6, 7].
// ---------------------------------------------------------------------------------------------------------------
constexpr int kLB = 256;

struct LongArgs {
  Batch b;
  Work w;
  WinOff W;
  int k, kl, T, J, n, m;
};

__device__ __forceinline__ double long_entry(const LongArgs& a, int r, int col) {  // K(r, col), 0 if absent
  const int32_t* kp = a.b.indptr + a.W.row;
  const int32_t* kc = a.b.indices + a.W.nz;
  const double* kv = a.b.data + a.W.nz;
  for (int p = kp[r]; p < kp[r + 1]; ++p)
    if (kc[p] == col) return kv[p];
  return 0.0;
}

__global__ __launch_bounds__(kLB) void long_init(LongArgs a) {
  const int t = blockIdx.x * kLB + threadIdx.x;
  if (t < a.n) a.w.dc[a.W.wn + t] = 1.0;
  if (t < a.m) a.w.dr[a.W.wm + t] = 1.0;
}

template <bool MAXR>
__global__ __launch_bounds__(kLB) void long_pass(LongArgs a) {
  const int t = blockIdx.x * kLB + threadIdx.x;
  const double* Dr = a.w.dr + a.W.wm;
  const double* Dc = a.w.dc + a.W.wn;
  auto acc_of = [](double acc, double v) { return MAXR ? fmax(acc, v) : acc + v; };
  if (t < a.m) {
    const int32_t* kp = a.b.indptr + a.W.row;
    const int32_t* kc = a.b.indices + a.W.nz;
    const double* kv = a.b.data + a.W.nz;
    double acc = 0.0;
    for (int p = kp[t]; p < kp[t + 1]; ++p) acc = acc_of(acc, fabs(kv[p]) * Dr[t] * Dc[kc[p]]);
    a.w.tmpr[a.W.wm + t] = acc > 0.0 ? 1.0 / sqrt(acc) : 1.0;
  }
  if (t < 3 * a.T) {
    const int T = a.T, v = t / T, st = t - v * T;
    const int32_t* dm = reinterpret_cast<const int32_t*>(a.w.vbuf + a.W.wn);
    const int r1 = v < 2 ? st + 1 : st, r2 = v < 2 ? dm[st] : st + 1;  // ascending rows
    double acc = fabs(long_entry(a, r1, t)) * Dc[t] * Dr[r1];
    if (r2 >= 0) acc = acc_of(acc, fabs(long_entry(a, r2, t)) * Dc[t] * Dr[r2]);
    a.w.tmpc[a.W.wn + t] = acc > 0.0 ? 1.0 / sqrt(acc) : 1.0;
  }
}

// one workgroup per tau column: its DCM rows in step order, partials per thread (strided), then in thread order
template <bool MAXR>
__global__ __launch_bounds__(kLB) void long_tau_pass(LongArgs a) {
  __shared__ double red[kLB];
  const int j = blockIdx.x, col = 3 * a.T + j, T = a.T;
  const double* Dr = a.w.dr + a.W.wm;
  const double* Dc = a.w.dc + a.W.wn;
  const int32_t* dm = reinterpret_cast<const int32_t*>(a.w.vbuf + a.W.wn);
  double acc = 0.0;
  for (int t = threadIdx.x; t < T; t += kLB) {
    if (dm[T + t] != j) continue;
    const int r = dm[t];
    const double v = fabs(long_entry(a, r, col)) * Dc[col] * Dr[r];
    acc = MAXR ? fmax(acc, v) : acc + v;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int u = 0; u < kLB; ++u) s = MAXR ? fmax(s, red[u]) : s + red[u];
    a.w.tmpc[a.W.wn + col] = s > 0.0 ? 1.0 / sqrt(s) : 1.0;
  }
}

__global__ __launch_bounds__(kLB) void long_apply(LongArgs a) {
  const int t = blockIdx.x * kLB + threadIdx.x;
  if (t < a.n) a.w.dc[a.W.wn + t] *= a.w.tmpc[a.W.wn + t];
  if (t < a.m) a.w.dr[a.W.wm + t] *= a.w.tmpr[a.W.wm + t];
}

// scaled data, reciprocal scalings, per-workgroup norm partials (wbuf scratch: [block][4])
__global__ __launch_bounds__(kLB) void long_fill(LongArgs a) {
  __shared__ double red[4 * (kLB / kWave)];
  const int t = blockIdx.x * kLB + threadIdx.x;
  const double* Dr = a.w.dr + a.W.wm;
  const double* Dc = a.w.dc + a.W.wn;
  double nrm[4] = {0.0, 0.0, 0.0, 0.0};  // ||cs||^2, ||qs||^2, ||c||^2, ||q||^2
  if (t < a.m) {
    const int32_t* kp = a.b.indptr + a.W.row;
    const int32_t* kc = a.b.indices + a.W.nz;
    const double* kv = a.b.data + a.W.nz;
    const double d = Dr[t];
    for (int p = kp[t]; p < kp[t + 1]; ++p) a.w.kval[a.W.wz + p] = kv[p] * d * Dc[kc[p]];
    const double qi = a.b.q[a.W.om + t];
    a.w.qs[a.W.wm + t] = qi * d;
    a.w.tmpr[a.W.wm + t] = 1.0 / d;
    nrm[1] = qi * d * qi * d;
    nrm[3] = qi * qi;
  }
  if (t < a.n) {
    const double cj = a.b.c[a.W.on + t], d = Dc[t];
    a.w.cs[a.W.wn + t] = cj * d;
    a.w.ls[a.W.wn + t] = a.b.l[a.W.on + t] / d;
    a.w.us[a.W.wn + t] = a.b.u[a.W.on + t] / d;
    a.w.tmpc[a.W.wn + t] = 1.0 / d;
    nrm[0] = cj * d * cj * d;
    nrm[2] = cj * cj;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 4; ++u) nrm[u] = wave_sum(nrm[u]);
  if (lane == 0)
#pragma unroll
    for (int u = 0; u < 4; ++u) red[4 * wid + u] = nrm[u];
  __syncthreads();
  if (threadIdx.x < 4) {
    double s = 0.0;
    for (int q = 0; q < kLB / kWave; ++q) s += red[4 * q + threadIdx.x];
    a.w.wbuf[a.W.wm + 4 * (int64_t)blockIdx.x + threadIdx.x] = s;
  }
}

__global__ __launch_bounds__(kLB) void long_norms(LongArgs a, int nblk, double step_safety) {
  __shared__ double red[4 * kLB];
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  for (int q = threadIdx.x; q < nblk; q += kLB)
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] += a.w.wbuf[a.W.wm + 4 * (int64_t)q + u];
#pragma unroll
  for (int u = 0; u < 4; ++u) red[4 * threadIdx.x + u] = v[u];
  __syncthreads();
  if (threadIdx.x == 0) {
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < kLB; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += red[4 * q + u];
    double* scal = a.w.scal + (int64_t)a.kl * kScal;
    const double ncs = sqrt(s[0]), nqs = sqrt(s[1]);
    scal[0] = step_safety;  // refined by the chain kernel's power iteration
    scal[1] = (ncs > 1e-10 && nqs > 1e-10) ? ncs / nqs : 1.0;
    scal[2] = sqrt(s[2]);
    scal[3] = sqrt(s[3]);
    scal[4] = scal[5] = 0.0;
    scal[6] = 0.0;
    scal[7] = 1.0;
  }
}

// ---------------------------------------------------------------------------------------------------------------
// The team kernel.
// ---------------------------------------------------------------------------------------------------------------
struct ChainArgs {
  const int32_t* pos;        // positions (into plan) of the windows to solve
  int npos;
  const int32_t* plan;
  unsigned long long* xbuf;  // NT * PT * kXSeg granules, zeroed before the launch
  int* abort_word;           // zeroed before the launch (with the diagnostics); [0] abort, [8] next window
  int PT, NT;
  int S;                     // workgroup slots per XCD (grid = 8 S)
  long long spin_ticks;      // longest wait for a partner's exchange (wall-clock ticks) before the launch aborts;
                             // < 0 (tests): abort at the first poll that has to wait
};

// Team and segment of workgroup b: blocks b and b + 8 share an XCD (round-robin dispatch, MI355X_MICROARCH.md --
// a speed assumption only, never a correctness one), so each XCD's first floor(S / PT) * PT slots form local
// teams and the remaining slots of all XCDs are pooled into further teams.  A team larger than an XCD (PT > S: the
// long windows) takes consecutive segments from one XCD's slots before the next XCD's, so only the few boundaries
// between XCDs hand off across L2s.  team >= NT: idle.
__host__ __device__ inline void chain_team_of(int b, int S, int PT, int* team, int* seg) {
  const int xcd = b % 8, slot = b / 8, LT = S / PT, used = LT * PT;
  if (PT > S) {
    const int li = xcd * S + slot;
    *team = li / PT;
    *seg = li % PT;
  } else if (slot < used) {
    *team = xcd * LT + slot / PT;
    *seg = slot % PT;
  } else {
    const int li = (slot - used) * 8 + xcd;
    *team = 8 * LT + li / PT;
    *seg = li % PT;
  }
}
__host__ __device__ inline int chain_teams(int S, int PT) {
  if (PT > S) return (8 * S) / PT;
  const int LT = S / PT;
  return 8 * LT + (8 * (S - LT * PT)) / PT;
}

__global__ __launch_bounds__(kCB, 3) void pdhg_chain_kernel(const Batch b, const Work w, const Chunk ch,
                                                           const Opts o, const ChainArgs a) {
  constexpr int B = kCB;
  constexpr int NW = B / kWave;
  constexpr int NC = 3, NR = 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int team, seg;
  chain_team_of((int)blockIdx.x, a.S, a.PT, &team, &seg);
  if (team >= a.NT) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* XE = reinterpret_cast<double*>(smem);  // x-bar of ene of the lane's step; [L] = next segment's first
  double* YS = XE + (B + 1);                     // y of row t0 + i; [0] = init row (segment 0) or the ghost row
  double* XT = YS + (B + 1);                     // x-bar of the tau slots
  double* XK = XT + kJSeg;                       // tau K'y totals of the KKT images
  double* GK = XK + kJSeg;                       // ghost row coefficients: ch, dis, ene of step t0 - 1, ene_t0
  double* red = GK + 4;
  double* TP = red + kNRed * (NW + 1) + 4;       // [kJSeg][B] per-lane partial K'y of the tau slots
  double* XP = TP + kJSeg * B;                   // [3][B] T(z) of the lane's columns (check iterations)
  double* YP = XP + NC * B;                      // [2][B] T(z) of the lane's rows
  double* CR = YP + NR * B;                      // [kPMax][kNRed] check partials of every segment
  double* RO = CR + kPMax * kNRed;               // [6][B]: c of ch, dis, ene; upper bound of ch, dis, ene
  int32_t* poff = reinterpret_cast<int32_t*>(smem + align16(sizeof(double) * chain_lds_doubles()));
  unsigned* pval = reinterpret_cast<unsigned*>(poff + kPollMax);
  // misc: [0] dead flag, [1] A entries, [2] K entries, [4] tau-image start in K,
  //       [8 + u] offset of slot u's partials relative to the tau start, [12 + u] / [16 + u] first / last segment
  //       sharing slot u's column
  int32_t* misc = poff + 2 * kPollMax;
  gu64* tb = (gu64*)a.xbuf + (int64_t)team * a.PT * kXSeg;  // the team's exchange area
  gi32* abort_word = (gi32*)a.abort_word;
  gu64* mine = tb + (int64_t)seg * kXSeg;

  if (tid == 0) misc[0] = 0;
  __syncthreads();
  for (int wseq = 1;; ++wseq) {
    // ---- the team's next window: segment 0 takes it from the launch-wide counter (after every segment has read
    //      the previous hand-out) and hands it to the others; every segment acknowledges
    if (wid == 0) {
      // one-granule entries of the C list area; bounded: the wait is limited in time (an acknowledgement); unbounded:
      // the next window's hand-out, which comes when segment 0 has finished its window (however long that takes --
      // segment 0 itself only waits in bounded polls, so it either hands out or aborts, and the abort word ends this)
      auto poll1 = [&](int e0, int cnt, unsigned tag, bool bounded) -> bool {
        const long long t0 = wall_clock64();
        for (int base = 0; base < cnt; base += kWave) {
          const bool act = base + lane < cnt;
          gu64* p = tb + (act ? poff[e0 + base + lane] : 0);
          bool ok = !act;
          unsigned spins = 0;
          while (!__all(ok)) {
            if (!ok) {
              const unsigned long long xv = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if ((unsigned)(xv >> 32) == tag) {
                ok = true;
                pval[e0 + base + lane] = (unsigned)xv;
              }
            }
            if ((++spins & 1023u) == 0 || a.spin_ticks < 0) {
              const bool late = bounded && wall_clock64() - t0 > a.spin_ticks;
              if (late || __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                if (lane == 0) {
                  __hip_atomic_store(abort_word + 16 + 8 * (int)blockIdx.x, late ? 3 : 2, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
                  __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                return false;
              }
            }
          }
        }
        return true;
      };
      const unsigned wtag = chain_tag(wseq, 0x3FFFF);  // round field all ones: no exchange round reaches it
      const int par = wseq & 1;
      bool ok = true;
      int wi = 0;
      if (seg == 0) {
        if (wseq > 1 && a.PT > 1) {  // acknowledgements of the previous hand-out
          for (int e = lane; e < a.PT - 1; e += kWave) poff[kPollC + e] = (e + 1) * kXSeg + kOffAck + (par ^ 1);
          __builtin_amdgcn_wave_barrier();
          ok = poll1(kPollC, a.PT - 1, chain_tag(wseq - 1, 0x3FFFF), true);
        }
        if (lane == 0) wi = __hip_atomic_fetch_add(abort_word + 8, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wi = __builtin_amdgcn_readfirstlane(wi);
        if (ok && lane == 0)
          __hip_atomic_store(tb + kOffW + par, ((unsigned long long)wtag << 32) | (unsigned)wi, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      } else {
        if (lane == 0) poff[kPollC] = kOffW + par;
        __builtin_amdgcn_wave_barrier();
        ok = poll1(kPollC, 1, wtag, false);
        wi = (int)pval[kPollC];
        if (ok && lane == 0)
          __hip_atomic_store(mine + kOffAck + par, ((unsigned long long)wtag << 32), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0) {
        misc[5] = wi;
        if (!ok) misc[0] = 1;
      }
    }
    __syncthreads();
    const int wi = misc[5];
    if (misc[0] || wi >= a.npos) break;
    const int32_t* pl = a.plan + (int64_t)a.pos[wi] * kPlanInts;
    const int P = pl[0];
    if (seg >= P) continue;
    const int T = pl[1], k = pl[3];
    const int t0 = pl[kPlanStart + seg], L = pl[kPlanStart + seg + 1] - t0;
    const bool first = seg == 0, last = seg == P - 1;
    const int kl = k - ch.first;
    const WinOff W = win_offsets(b, ch, k);
    const int n = W.n;
    const double* scal = w.scal + (int64_t)kl * kScal;
    int nsl = 0;
#pragma unroll
    for (int u = 0; u < kJSeg; ++u) nsl += pl[kPlanSlot + 4 * seg + u] >= 0;
    const int wl = (L - 1) >> 6;  // wave holding the segment's last step
    const int32_t* gkp = b.indptr + W.row;
    const int32_t* gkc = b.indices + W.nz;
    const double* gkv = w.kval + W.wz;
    const double* cs = w.cs + W.wn;
    const double* ls = w.ls + W.wn;
    const double* us = w.us + W.wn;
    const double* qs = w.qs + W.wm;
    const double* dcv = w.dc + W.wn;
    const double* drv = w.dr + W.wm;
    const int32_t* dm = reinterpret_cast<const int32_t*>(w.vbuf + W.wn);
    double* xo_g = b.x + W.on;
    double* yo_g = b.y + W.om;
    int cA = 0, cB = 0, cK = 0, cC = 0;  // rounds of each exchange kind (identical in every segment and wave)
#ifdef DVH_CHAIN_PROBE_TIMING
    long long t_probe[2] = {0, 0};  // wave 0's waits: tau partials, boundary (timing probe builds only)
#endif

    // ---- poll lists (offset at parity 0 in the low 16 bits, parity stride above): A = the tau partials of the
    //      other segments sharing a slot (by slot, then segment); K = {first-ene image from s+1} + tau image
    //      partials; up = ch, dis, ene of s-1's last step; down = s+1's first ene
    if (tid == 0) {
      int e = 0, ek = kPollK;
      if (!last) {
        poff[ek++] = ((seg + 1) * kXSeg + kOffK) | (12 << 16);
        poff[ek++] = ((seg + 1) * kXSeg + kOffK + 1) | (12 << 16);
        poff[kPollD] = ((seg + 1) * kXSeg + kOffD) | (2 << 16);
        poff[kPollD + 1] = ((seg + 1) * kXSeg + kOffD + 1) | (2 << 16);
      }
      if (!first)
        for (int g = 0; g < 6; ++g) poff[kPollU + g] = ((seg - 1) * kXSeg + kOffU + g) | (6 << 16);
      misc[4] = ek - kPollK;
      int rel = 0;
      for (int u = 0; u < nsl; ++u) {
        const int id = pl[kPlanSlot + 4 * seg + u], rlo = pl[kPlanLo + 4 * seg + u], rhi = pl[kPlanHi + 4 * seg + u];
        misc[8 + u] = rel;
        misc[12 + u] = rlo;
        misc[16 + u] = rhi;
        for (int r = rlo; r <= rhi; ++r) {
          if (r == seg) continue;
          int ur = 0;
          while (ur < kJSeg - 1 && pl[kPlanSlot + 4 * r + ur] != id) ++ur;
          poff[e++] = (r * kXSeg + kOffA2 + 2 * ur) | (8 << 16);
          poff[e++] = (r * kXSeg + kOffA2 + 2 * ur + 1) | (8 << 16);
          poff[ek++] = (r * kXSeg + kOffK + 2 + 2 * ur) | (12 << 16);
          poff[ek++] = (r * kXSeg + kOffK + 3 + 2 * ur) | (12 << 16);
          rel += 2;
        }
      }
      misc[1] = e;
      misc[2] = ek - kPollK;
    }
    __syncthreads();
    const int nA = misc[1], nK = misc[2], kTau = misc[4];

    // polls entries [e0, e0 + cnt) for round c (tag, parity); the 32-bit halves land in pval[e0 ..]; false: the
    // wait outlasted spin_ticks or another workgroup aborted (the abort word is then set)
    auto poll = [&](int e0, int cnt, int c) -> bool {
      const unsigned tag = chain_tag(wseq, c);
      const int par = c & 1;
      const long long tw = wall_clock64();
      for (int base = 0; base < cnt; base += kWave) {
        const int e = base + lane;
        const bool act = e < cnt;
        const int ent = act ? poff[e0 + e] : 0;
        gu64* p = tb + (ent & 0xFFFF) + par * (ent >> 16);
        bool ok = !act;
        unsigned v = 0, seen = 0;
        unsigned spins = 0;
        while (true) {
          if (!ok) {
            const unsigned long long xv = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            seen = (unsigned)(xv >> 32);
            if (seen == tag) {
              ok = true;
              v = (unsigned)xv;
            }
          }
          if (__all(ok)) break;
#ifdef DVH_CHAIN_POLL_SLEEP
          __builtin_amdgcn_s_sleep(DVH_CHAIN_POLL_SLEEP);
#endif
          ++spins;
          bool late = false;
          if (((spins & 1023u) == 0 || a.spin_ticks < 0) && ((late = wall_clock64() - tw > a.spin_ticks) ||
                                       __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            // diagnostics per workgroup (abort_word[16 + 8 blockIdx]): {1 = timed out / 2 = saw the abort, list
            // start, round, entry, expected tag, tag seen}
            const unsigned long long bad = __ballot(!ok);
            const int fl = bad ? __ffsll((long long)bad) - 1 : 0;
            if (lane == fl) {
              const int d[6] = {late ? 1 : 2, e0, c, ent, (int)tag, (int)seen};
              for (int u = 0; u < 6; ++u)
                __hip_atomic_store(abort_word + 16 + 8 * (int)blockIdx.x + u, d[u], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            if (lane == 0) __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
          }
        }
        if (act) pval[e0 + e] = v;
      }
      return true;
    };
    auto pv64 = [&](int e) { return __hiloint2double((int)pval[e], (int)pval[e + 1]); };
    // tau total of slot u from this segment's partial and the polled ones (entries at e0 + rel[u] ..), the same
    // additions in every segment holding the slot's rows: lane i holds the partial of segment rlo + i and the wave sums
    // them with one fixed DPP tree (lane 0's result), so every sharer gets the same bits.  (Summed one after another in
    // segment order, the ~12 dependent LDS reads and adds of a 5-minute month sat on wave 0's critical path.)
    auto tau_total = [&](int u, double own, int e0) -> double {
      const int rlo = misc[12 + u], rhi = misc[16 + u];
      if (rhi - rlo < kWave) {
        const int r = rlo + lane, base = e0 + misc[8 + u];
        double v = 0.0;
        if (r <= rhi) v = r == seg ? own : pv64(base + 2 * (r < seg ? lane : lane - 1));
        return uniform(wave_sum_dpp(v));
      }
      int e = e0 + misc[8 + u];
      double s = 0.0;
      for (int r = rlo; r <= rhi; ++r) {
        if (r == seg) {
          s += own;
        } else {
          s += pv64(e);
          e += 2;
        }
      }
      return s;
    };

    // ---- the lane's step t = t0 + tid
    const int t = t0 + tid;
    const bool val = tid < L;
    auto col = [&](int v) { return v * T + t; };
    double x[NC], xa[NC];
    double loe = 0.0;
    double ks[4] = {0.0, 0.0, 0.0, 0.0};  // SOE row of step t: ch_t, dis_t, ene_t, ene_{t+1}
    double kd[3] = {0.0, 0.0, 0.0};       // DCM row of step t: ch_t, dis_t, tau
    double kp = 0.0;                      // ene_t in row t (init row, or the previous step's SOE row)
    double y[NR], ya[NR], q[2];
    int drow = -1, jt = 0;
#pragma unroll
    for (int v = 0; v < NC; ++v) {
      x[v] = xa[v] = 0.0;
      RO[v * B + tid] = RO[(NC + v) * B + tid] = 0.0;
    }
    auto cof = [&](int v) -> double { return RO[v * B + tid]; };
    auto hib = [&](int v) -> double { return RO[(NC + v) * B + tid]; };
#pragma unroll
    for (int r = 0; r < NR; ++r) y[r] = ya[r] = 0.0;
    q[0] = q[1] = 0.0;
    if (val) {
#pragma unroll
      for (int v = 0; v < NC; ++v) {
        const int j = col(v);
        RO[(NC + v) * B + tid] = us[j];
        RO[v * B + tid] = cs[j];
        x[v] = xa[v] = fmin(fmax(0.0, ls[j]), us[j]);
      }
      loe = ls[2 * T + t];
      for (int p = gkp[t + 1]; p < gkp[t + 2]; ++p) {
        const int c = gkc[p];
        const double av = gkv[p];
        if (c == t) ks[0] = av;
        else if (c == T + t) ks[1] = av;
        else if (c == 2 * T + t) ks[2] = av;
        else ks[3] = av;
      }
      for (int p = gkp[t]; p < gkp[t + 1]; ++p)
        if (gkc[p] == 2 * T + t) kp = gkv[p];
      q[0] = qs[t + 1];
      drow = dm[t];
      if (drow >= 0) {
        const int jg = dm[T + t];
#pragma unroll
        for (int u = 0; u < kJSeg; ++u)
          if (pl[kPlanSlot + 4 * seg + u] == jg) jt = u;
        for (int p = gkp[drow]; p < gkp[drow + 1]; ++p) {
          const int c = gkc[p];
          const double av = gkv[p];
          if (c < T) kd[0] = av;
          else if (c < 2 * T) kd[1] = av;
          else kd[2] = av;
        }
        q[1] = qs[drow];
      }
      if (o.warm) {
#pragma unroll
        for (int v = 0; v < NC; ++v) {
          const int j = col(v);
          x[v] = xa[v] = fmin(fmax(xo_g[j] / dcv[j], ls[j]), us[j]);
        }
        y[0] = ya[0] = yo_g[t + 1] / drv[t + 1];
        if (drow >= 0) y[1] = ya[1] = fmax(yo_g[drow] / drv[drow], 0.0);
      }
    }
    const int xta = lds_addr(XT + jt);
    // wave 0 special lanes: u < nsl the tau slots {x, xa, c, lo, hi, x+}; the last lane the row of YS[0]: the
    // init row (segment 0: {y, ya, y+, q, coefficient}) or the ghost boundary row ({y, ya, y+, q}, GK)
    constexpr int kRowLane = kWave - 1;
    static_assert(kJSeg < kRowLane, "tau lanes and the row lane are distinct");
    // the tau slots live in wave kTauWave, the init / ghost row in wave 0: their serial work (the tau partials'
    // reduction, exchange and update; the ghost row's boundary poll and dual step) runs in two waves side by side
    const bool tlane = wid == kTauWave && lane < nsl, rlane = wid == 0 && lane == kRowLane;
    const bool ilane = rlane && first, glane = rlane && !first;
    int jg0 = 0;
    bool town = false;  // this segment owns the slot (the lowest segment holding its rows): KKT / norm terms
    if (tlane) {
      jg0 = pl[kPlanSlot + 4 * seg + lane];
      town = pl[kPlanLo + 4 * seg + lane] == seg;
    }
    double sp[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (tlane) {
      const double l0 = ls[3 * T + jg0], h0 = us[3 * T + jg0];
      sp[0] = sp[1] = sp[5] = fmin(fmax(0.0, l0), h0);
      sp[2] = cs[3 * T + jg0];
      sp[3] = l0;
      sp[4] = h0;
      if (o.warm) sp[0] = sp[1] = sp[5] = fmin(fmax(xo_g[3 * T + jg0] / dcv[3 * T + jg0], l0), h0);
    }
    if (ilane) {
      sp[3] = qs[0];
      sp[4] = gkv[gkp[0]];
      if (o.warm) sp[0] = sp[1] = sp[2] = yo_g[0] / drv[0];
    }
    if (glane) {  // row t0 = SOE row of step t0 - 1 (owned by segment s - 1)
      double g4[4] = {0.0, 0.0, 0.0, 0.0};
      for (int p = gkp[t0]; p < gkp[t0 + 1]; ++p) {
        const int c = gkc[p];
        const double av = gkv[p];
        if (c == t0 - 1) g4[0] = av;
        else if (c == T + t0 - 1) g4[1] = av;
        else if (c == 2 * T + t0 - 1) g4[2] = av;
        else g4[3] = av;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) GK[u] = g4[u];
      sp[3] = qs[t0];
      if (o.warm) sp[0] = sp[1] = yo_g[t0] / drv[t0];
    }
    if (tid < kJSeg) XT[tid] = XK[tid] = 0.0;
    if (tid == 0) XE[B] = YS[B] = 0.0;
    XE[tid] = YS[tid] = 0.0;
    for (int u = tid; u < kJSeg * B; u += B) TP[u] = 0.0;
#pragma unroll
    for (int v = 0; v < NC; ++v) XP[v * B + tid] = x[v];
#pragma unroll
    for (int r = 0; r < NR; ++r) YP[r * B + tid] = y[r];
    __syncthreads();

    // ---- SpMV pieces (as dvh_band.hip)
    auto ktr = [&](const double (&vr)[NR], double vprev, double (&out)[NC]) {
      out[0] = fma(kd[0], vr[1], ks[0] * vr[0]);
      out[1] = fma(kd[1], vr[1], ks[1] * vr[0]);
      out[2] = fma(ks[2], vr[0], kp * vprev);
    };
    auto kown = [&](const double (&v)[NC], double (&os)[NR]) {
      os[0] = fma(ks[2], v[2], fma(ks[1], v[1], ks[0] * v[0]));
      os[1] = fma(kd[1], v[1], kd[0] * v[0]);
    };
    auto kfin = [&](double (&os)[NR], double vnext) {
      os[0] = fma(ks[3], vnext, os[0]);
      os[1] = fma(kd[2], lds_ld(xta), os[1]);
    };
    // the ghost row's K v from s-1's last step (polled, up) and v of ene_t0: the owner's kown + kfin, same order
    auto kghost = [&]() -> double {
      const double v0 = pv64(kPollU), v1 = pv64(kPollU + 2), v2 = pv64(kPollU + 4);
      return fma(GK[3], XE[0], fma(GK[2], v2, fma(GK[1], v1, GK[0] * v0)));
    };
    auto tau_parts = [&](double vd) {
      if (nsl == 1) {
        TP[tid] = kd[2] * vd;
      } else {
        for (int j = 0; j < nsl; ++j) TP[j * B + tid] = (jt == j ? kd[2] : 0.0) * vd;
      }
    };
    // wave 0: lane u < nsl gets this segment's partial sum of TP[u][.] (fixed order)
    auto tau_own = [&]() {
      double res = 0.0;
      for (int j = 0; j < nsl; ++j) {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < NW; ++r) s += TP[j * B + r * kWave + lane];
        s = uniform(wave_sum_dpp(s));
        if (lane == j) res = s;
      }
      return res;
    };
    // wave 0: publish this segment's tau partials for round cA (before its primal work) ...
    auto publish_a = [&](double own) {
      if (lane < nsl) put_f64(mine + kOffA2 + 8 * (cA & 1) + 2 * lane, chain_tag(wseq, cA), own);
    };
    // ... and, after it, collect the sharers' and return the totals (lanes u < nsl); false in ok: abort
    auto collect_a = [&](double own, bool& ok) -> double {
#ifdef DVH_CHAIN_PROBE_NO_TAU_XCHG  // timing probe only (wrong results): the segment's own partials as the totals
      return own;
#endif
#ifdef DVH_CHAIN_PROBE_TIMING
      const long long c0_ = wall_clock64();
      const bool pok_ = poll(0, nA, cA);
      t_probe[0] += wall_clock64() - c0_;
      if (!pok_) {
#else
      if (!poll(0, nA, cA)) {
#endif
        ok = false;
        return 0.0;
      }
      double tot = 0.0;
      for (int u = 0; u < nsl; ++u) {
        const double tu = tau_total(u, readlane_f64(own, u), 0);
        if (lane == u) tot = tu;
      }
      return tot;
    };
    // after the primal half-step: the first ene goes down (lane 0), the last step's ch, dis, ene go up (lane L-1)
    auto publish_b = [&](const double (&v)[NC]) {
      const unsigned tag = chain_tag(wseq, cB);
      if (!first && tid == 0) put_f64(mine + kOffD + 2 * (cB & 1), tag, v[2]);
      if (!last && tid == L - 1) {
        gu64* g = mine + kOffU + 6 * (cB & 1);
        put_f64(g, tag, v[0]);
        put_f64(g + 2, tag, v[1]);
        put_f64(g + 4, tag, v[2]);
      }
    };
    // before the dual half-step: wave wl takes the next segment's first ene into XE[L]; wave 0 the previous
    // segment's last step (for the ghost row, in pval[kPollU ..]).  Sets the dead flag on an abort.
    auto poll_b = [&]() {
#ifdef DVH_CHAIN_PROBE_NO_HOP  // timing probe only (wrong results): no boundary exchange
      return;
#endif
      if (!last && wid == wl) {
        if (poll(kPollD, 2, cB)) {
          if (lane == 0) XE[L] = pv64(kPollD);
        } else if (lane == 0) {
          misc[0] = 1;
        }
      }
#ifdef DVH_CHAIN_PROBE_TIMING
      const long long c0_ = wall_clock64();
#endif
      if (!first && wid == 0 && !poll(kPollU, 6, cB) && lane == 0) misc[0] = 1;
#ifdef DVH_CHAIN_PROBE_TIMING
      t_probe[1] += wall_clock64() - c0_;
#endif
    };
    // check reduction: this segment's NV partials (identical in every lane on entry) -> the sums over all segments
    // in segment order, in every lane; false: abort.  A leader reduction: every other segment publishes its partials,
    // segment 0 collects them with all its waves (P - 1 segments x NV values: one or two polls per thread even for
    // the 137 segments of a 5-minute annual window), sums them in segment order and publishes the totals, which the
    // others poll -- two hops, but O(P) loads in total instead of O(P^2), and every segment gets the same bits.
    auto round_c = [&](auto& acc) -> bool {
      constexpr int nv = sizeof(acc) / sizeof(double);
      ++cC;
      const int par = cC & 1;
      const unsigned tag = chain_tag(wseq, cC);
      double mv = 0.0;
#pragma unroll
      for (int v = 0; v < nv; ++v)
        if (lane == v) mv = acc[v];
      if (first) {
        if (wid == 0 && lane < nv) CR[lane] = mv;
        const int cnt = (P - 1) * nv;
        const long long tw = wall_clock64();
        for (int base = 0; base < cnt; base += B) {
          const int i = base + tid;
          const bool act = i < cnt;
          const int r = act ? 1 + i / nv : 0, v = act ? i % nv : 0;
          gu64* g = tb + (int64_t)r * kXSeg + kOffC + kCW * par + 2 * v;
          bool ok = !act;
          unsigned hi = 0, lo = 0, spins = 0;
          while (!__all(ok)) {
            if (!ok) {
              const unsigned long long a0 = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const unsigned long long a1 = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if ((unsigned)(a0 >> 32) == tag && (unsigned)(a1 >> 32) == tag) {
                ok = true;
                hi = (unsigned)a0;
                lo = (unsigned)a1;
              }
            }
            bool late = false;
            if (((++spins & 1023u) == 0 || a.spin_ticks < 0) && ((late = wall_clock64() - tw > a.spin_ticks) ||
                                           __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
              if (lane == 0) {
                const int d[6] = {late ? 1 : 2, -1, cC, r, (int)tag, 0};
                for (int u = 0; u < 6; ++u)
                  __hip_atomic_store(abort_word + 16 + 8 * (int)blockIdx.x + u, d[u], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                misc[0] = 1;
              }
              break;
            }
          }
          if (act && ok) CR[r * kNRed + v] = __hiloint2double((int)hi, (int)lo);
          if (misc[0]) break;
        }
        lds_barrier();
        if (wid == 0 && lane < nv && !misc[0]) {
          double s = 0.0;
          for (int r = 0; r < P; ++r) s += CR[r * kNRed + lane];
          put_f64(tb + kOffT + kCW * par + 2 * lane, tag, s);
          CR[lane] = s;
        }
      } else if (wid == 0) {
        if (lane < nv) put_f64(mine + kOffC + kCW * par + 2 * lane, tag, mv);
        if (lane < 2 * nv) poff[kPollC + lane] = (kOffT + lane) | (kCW << 16);
        __builtin_amdgcn_wave_barrier();
        if (!poll(kPollC, 2 * nv, cC)) {
          if (lane == 0) misc[0] = 1;
        } else if (lane < nv) {
          CR[lane] = pv64(kPollC + 2 * lane);
        }
      }
      lds_barrier();
      if (misc[0]) return false;
#pragma unroll
      for (int v = 0; v < nv; ++v) acc[v] = CR[v];
      lds_barrier();  // CR is rewritten by the next reduction
      return true;
    };

    // ---- ||Kt||_2 by power iteration (as the band kernel, exchanging across the segment boundaries)
    double eta = scal[0];
    bool alive = true;
    {
      const int PI = o.power_iters;
      const double v0 = 1.0 / sqrt((double)n);
      double vc[NC];
#pragma unroll
      for (int v = 0; v < NC; ++v) vc[v] = val ? v0 : 0.0;
      double vtau = tlane ? v0 : 0.0;
      double nv[2] = {0.0, 0.0};
      double wr[NR] = {0.0, 0.0};
      for (int pi = 0; pi <= PI; ++pi) {
        if (pi > 0) {
          ++cA;
          if (wid == kTauWave) {
            const double own = tau_own();
            publish_a(own);
            bool ok = true;
            const double kt = collect_a(own, ok);
            if (!ok && lane == 0) misc[0] = 1;
            if (tlane) vtau = kt;
          }
          ktr(wr, YS[tid], vc);
        }
        if (pi >= PI - 1) {
          double s = town ? vtau * vtau : 0.0;
#pragma unroll
          for (int v = 0; v < NC; ++v) s = fma(vc[v], vc[v], s);
          nv[pi - (PI - 1)] = s;
        }
        if (pi == PI) break;
        XE[tid] = vc[2];
        if (tlane) XT[lane] = vtau;
        ++cB;
        publish_b(vc);
        lds_barrier();
        if (misc[0]) {
          alive = false;
          break;
        }
        poll_b();
        kown(vc, wr);
        kfin(wr, XE[tid + 1]);
        YS[tid + 1] = wr[0];
        if (ilane) YS[0] = sp[4] * XE[0];
        if (glane) YS[0] = kghost();
        if (nsl > 0) tau_parts(wr[1]);
        lds_barrier();
        if (misc[0]) {
          alive = false;
          break;
        }
      }
      if (alive) {
        lds_barrier();
        if (misc[0]) alive = false;
      }
      if (alive) {
        block_sum<B, 2>(nv, red);
        alive = round_c(nv);
        if (alive && nv[0] > 0.0 && nv[1] > 0.0) eta = o.step_safety / sqrt(sqrt(nv[1] / nv[0]));
      }
      YS[tid] = 0.0;
      if (tid == 0) YS[B] = 0.0;
      for (int u = tid; u < kJSeg * B; u += B) TP[u] = 0.0;
      __syncthreads();
    }
    if (!alive) break;
    // y images of the starting point (YS, TP)
    if (val) YS[tid + 1] = y[0];
    if (rlane) YS[0] = sp[0];
    if (nsl > 0) tau_parts(y[1]);
    __syncthreads();

    eta = uniform(eta);
    double pw = uniform(scal[1]);
    const double cnorm = uniform(scal[2]), qnorm = uniform(scal[3]), c0 = uniform(b.c0[k]);
    int it = 0, kin = 0, status = kIterLimit;
    double r0 = -1.0, rprev = -1.0;
    double fin[4] = {NAN, NAN, NAN, NAN};
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
    double kx[NR];  // own-column part of K x-bar for the dual half-step

    auto iterate = [&](auto chk_tag) __attribute__((always_inline)) {
      constexpr bool CHECK = decltype(chk_tag)::value;
      if (kin - kbase >= kWave) {
        kbase = kin;
        hw = hload(kin);
      }
      const double cb = readlane_f64(hw, kin - kbase), ca = 1.0 - cb;
      mv0 = mv1 = mv2 = mv3 = 0.0;
      ++cA;
      ++cB;
      // the tau columns' update: wave 0 collects the sharers' partials and updates the columns it holds.  The partials
      // go out at the start of the primal half-step; the collection waits in the dual half-step, beside the boundary
      // hop's, so the two exchanges' latencies overlap (one extra LDS barrier makes the columns' x-bar visible before
      // the DCM rows use them).  In the primal half-step instead, the tau exchange stood in front of the boundary hop:
      // 5.3 us per config-3 DCM iteration, of which 2.5 us the tau exchange (profiles/r04b_chain_anatomy.log).
      auto tau_step = [&](double own) {
        bool ok = true;
        const double kt = collect_a(own, ok);
        if (!ok && lane == 0) misc[0] = 1;
        if (tlane) {
          const double xo = sp[0], xan = sp[1];
          const double p1 = vmin(vmax(fma(-tau, sp[2] - kt, xo), sp[3]), sp[4]);
          const double xbt = fma(2.0, p1, -xo);
          XT[lane] = xbt;
          sp[0] = fma(ca, xbt, cb * xan);
          if (CHECK) {
            if (town) {
              const double d = xo - p1, da = p1 - xan;
              mv0 += d * d;
              mv1 += da * da;
            }
            sp[5] = p1;
          }
        }
      };
      double own = 0.0;
      // (DVH_CHAIN_PRIO) the waves whose primal work ends in a hand-off -- the tau wave's partials, wave 0's first ene
      // (down), the last step's wave (up) -- issue first on their SIMDs until they have published
      const bool hot = DVH_CHAIN_PRIO && (wid == kTauWave || wid == 0 || wid == wl);
      if (hot) __builtin_amdgcn_s_setprio(DVH_CHAIN_PRIO);
      // ---------------- primal half-step (reflected Halpern, rho = 1)
      {
        if (wid == kTauWave) {
          own = tau_own();
          publish_a(own);
        }
        double kty[NC], xb[NC];
        ktr(y, YS[tid], kty);
#pragma unroll
        for (int v = 0; v < NC; ++v) {  // padding steps have c = lo = hi = 0 and stay at 0
          const double lo = v == 2 ? loe : 0.0;
          const double p1 = vmin(vmax(fma(-tau, cof(v) - kty[v], x[v]), lo), hib(v));
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
        publish_b(xb);
        if (hot) __builtin_amdgcn_s_setprio(0);
        kown(xb, kx);
#ifdef DVH_CHAIN_TAU_IN_PRIMAL  // A/B: the round-3 placement
        if (wid == kTauWave) tau_step(own);
#endif
      }
      lds_barrier();
      // ---------------- dual half-step
      {
        poll_b();
#ifndef DVH_CHAIN_TAU_IN_PRIMAL
        if (nsl > 0) {  // uniform over the workgroup: the segment holds tau columns
          if (wid == kTauWave) tau_step(own);
          lds_barrier();
        }
#endif
        kfin(kx, XE[tid + 1]);
#pragma unroll
        for (int r = 0; r < NR; ++r) {  // row 0 (SOE) is an equality; the DCM row is >=: its dual stays >= 0
          double p1 = fma(sigma, q[r] - kx[r], y[r]);
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
        if (nsl > 0) tau_parts(y[1]);
        if (rlane) {  // init row (segment 0: ene_0 = target) or the ghost boundary row (counted by its owner)
          const double y0 = sp[0], ya0 = sp[1];
          const double q1 = first ? fma(sigma, sp[3] - sp[4] * XE[0], y0) : fma(sigma, sp[3] - kghost(), y0);
          if (CHECK) {
            if (first) {
              const double d = y0 - q1, da = q1 - ya0;
              mv2 += d * d;
              mv3 += da * da;
            }
            sp[2] = q1;
          }
          const double yn = fma(ca, fma(2.0, q1, -y0), cb * ya0);
          sp[0] = yn;
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
        if (misc[0]) break;
        continue;
      }
      ck = chk;
      iterate(Tt());
      if (misc[0]) break;
      // ---------------- check (as the band kernel), over the whole window
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
        // (DVH_CHAIN_KKT_PREFETCH) the lane's factors first, branch-free (a padding step / absent row loads entry 0 and
        // discards it), from indices formed here from an opaque thread index: they arrive during the exchange below
        double dcl[NC], drl[NR], dspl = 1.0;
        if constexpr (DVH_CHAIN_KKT_PREFETCH) {
          const int to = opaque(tid);
          const bool vo = to < L;
          const int tg = t0 + to;  // (this segment's first step + the lane)
#pragma unroll
          for (int v = 0; v < NC; ++v) {
            const double dv = dcv[vo ? v * T + tg : 0];
            dcl[v] = vo ? dv : 1.0;
          }
          const double d0 = drv[vo ? tg + 1 : 0];
          drl[0] = vo ? d0 : 1.0;
          const double d1 = drv[drow >= 0 ? drow : 0];
          drl[1] = drow >= 0 ? d1 : 1.0;
          const double dt_ = dcv[tlane ? 3 * T + jg0 : 0], di_ = drv[0];
          dspl = tlane ? dt_ : ilane ? di_ : 1.0;
        }
        // images of T(z_k); the next segment's first-ene image and the tau image totals come by exchange (the
        // ghost row's image is local)
        double xp[NC], yp[NR];
#pragma unroll
        for (int v = 0; v < NC; ++v) xp[v] = XP[v * B + tid];
#pragma unroll
        for (int r = 0; r < NR; ++r) yp[r] = YP[r * B + tid];
        XE[tid] = xp[2];
        YS[tid + 1] = yp[0];
        if (rlane) YS[0] = sp[2];
        if (tlane) XT[lane] = sp[5];
        if (nsl > 0) tau_parts(yp[1]);
        lds_barrier();
        if (wid == 0) {
          ++cK;
          const unsigned tag = chain_tag(wseq, cK);
          gu64* g = mine + kOffK + 12 * (cK & 1);
          const double own = tau_own();
          if (lane == 0 && !first) put_f64(g, tag, XE[0]);
          if (lane < nsl) put_f64(g + 2 + 2 * lane, tag, own);
          if (!poll(kPollK, nK, cK)) {
            if (lane == 0) misc[0] = 1;
          } else {
            if (!last && lane == 0) XE[L] = pv64(kPollK);
            double tot = 0.0;
            for (int u = 0; u < nsl; ++u) {
              const double tu = tau_total(u, readlane_f64(own, u), kPollK + kTau);
              if (lane == u) tot = tu;
            }
            if (lane < nsl) XK[lane] = tot;
          }
        }
        lds_barrier();
        if (misc[0]) break;
        auto col_kkt = [&](int j, double kt, double cj, double loj, double hij, double xj, double dpre) {
          const ColKktC r = col_kkt_c(kt, cj, loj, hij, xj, DVH_CHAIN_KKT_PREFETCH ? dpre : dcv[opaque(j)]);
          acc[5] += r.rd2;
          acc[6] += r.cx;
          acc[8] += r.bt;
          if (DVH_KKT_RDX) acc[kRdx] += r.rdx;
        };
        auto row_kkt = [&](int i, double kv, double qi, double yi, bool ge, double dpre) {
          const RowKktC r = row_kkt_c(kv, qi, yi, DVH_CHAIN_KKT_PREFETCH ? dpre : drv[opaque(i)], ge);
          acc[4] += r.rp2;
          acc[7] += qi * yi;
          acc[9] += r.y2;
        };
        double kt[NC];
        ktr(yp, YS[tid], kt);
        if (val) {
#pragma unroll
          for (int v = 0; v < NC; ++v) col_kkt(col(v), kt[v], cof(v), v == 2 ? loe : 0.0, hib(v), xp[v], dcl[v]);
        }
        if (tlane && town) col_kkt(3 * T + jg0, XK[lane], sp[2], sp[3], sp[4], sp[5], dspl);
        double kv[NR];
        kown(xp, kv);
        kfin(kv, XE[tid + 1]);
        if (val) row_kkt(t + 1, kv[0], q[0], yp[0], false, drl[0]);
        if (drow >= 0) row_kkt(drow, kv[1], q[1], yp[1], true, drl[1]);
        if (ilane) row_kkt(0, sp[4] * XE[0], sp[3], sp[2], false, dspl);
      }
      if (kkt) {
        block_sum1<B, kNRed, true>(acc, red);
        if (!round_c(acc)) break;
      } else {
        double acc4[4] = {acc[0], acc[1], acc[2], acc[3]};
        block_sum1<B, 4, true>(acc4, red);
        if (!round_c(acc4)) break;
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = acc4[u];
      }
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
        if (ddx > 1e-10 && ddy > 1e-10) pw = uniform(pw_update(ddy / ddx, pw, o.theta));
        tau = uniform(eta / pw);
        sigma = uniform(eta * pw);
#pragma unroll
        for (int v = 0; v < NC; ++v) x[v] = xa[v] = XP[v * B + tid];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) y[rr] = ya[rr] = YP[rr * B + tid];
        if (rlane) sp[0] = sp[1] = sp[2];
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
        if (rlane) YS[0] = sp[0];
        if (nsl > 0) tau_parts(y[1]);
      }
      lds_barrier();
    }
    if (misc[0]) break;
    // outputs: the last check's T(z_k), unscaled
    if (val) {
#pragma unroll
      for (int v = 0; v < NC; ++v) xo_g[col(v)] = XP[v * B + tid] * dcv[col(v)];
      yo_g[t + 1] = YP[tid] * drv[t + 1];
      if (drow >= 0) yo_g[drow] = YP[B + tid] * drv[drow];
    }
    if (tlane && town) xo_g[3 * T + jg0] = sp[5] * dcv[3 * T + jg0];
    if (ilane) yo_g[0] = sp[2] * drv[0];
#ifdef DVH_CHAIN_PROBE_TIMING
    if (tid == kTauWave * kWave) abort_word[16 + 8 * (int)blockIdx.x + 6] = (int)t_probe[0];
    if (tid == 0) abort_word[16 + 8 * (int)blockIdx.x + 7] = (int)t_probe[1];
#endif
    if (first && tid == 0) {
      b.istats[2 * k] = status;
      b.istats[2 * k + 1] = it;
      for (int u = 0; u < 4; ++u) b.stats[4 * k + u] = fin[u];
    }
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_chain_plan(const Batch& b, const Work& w, const Chunk& ch, const int32_t* list, int nlist,
                             int max_T, int32_t* plan, hipStream_t s) {
  (void)max_T;
  const size_t lds = sizeof(int32_t) * ((size_t)kRunsLds + 1);  // run starts
  hipError_t e = hipFuncSetAttribute((const void*)chain_plan_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(chain_plan_kernel, dim3(nlist), dim3(kPlanB), lds, s, b, w, ch, list, plan);
  return hipGetLastError();
}

hipError_t chain_capacity(int device, int* blocks) {
  const size_t lds = chain_lds_bytes();
  hipError_t e = hipFuncSetAttribute((const void*)pdhg_chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  int per_cu = 0, cus = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)pdhg_chain_kernel, kCB, lds);
  if (e != hipSuccess) return e;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return e;
  *blocks = per_cu * cus;
  return hipSuccess;
}

size_t chain_abort_bytes(int S) { return sizeof(int32_t) * (16 + 64 * (size_t)S); }
size_t chain_xbuf_bytes(int NT, int PT) { return sizeof(unsigned long long) * (size_t)NT * PT * kXSeg; }

int chain_team_count(int S, int PT) { return chain_teams(S, PT); }

hipError_t launch_chain(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, const int32_t* pos, int npos,
                        const int32_t* plan, int PT, int S, void* xbuf, int32_t* abort_word, long long spin_ticks,
                        hipStream_t s) {
  if (npos > 0x3FFF - 1) return hipErrorInvalidValue;  // window tags keep 14 bits of a team's window count
  const int NT = chain_teams(S, PT);
  const size_t lds = chain_lds_bytes();
  hipError_t e = hipFuncSetAttribute((const void*)pdhg_chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(xbuf, 0, chain_xbuf_bytes(NT, PT), s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(abort_word, 0, chain_abort_bytes(S), s);
  if (e != hipSuccess) return e;
  ChainArgs a{pos, npos, plan, static_cast<unsigned long long*>(xbuf), abort_word, PT, NT, S, spin_ticks};
  Batch bb = b;
  Work ww = w;
  Chunk cc = ch;
  Opts oo = o;
  void* args[] = {&bb, &ww, &cc, &oo, &a};
  // An ordinary launch of the capacity-sized grid (chain_capacity: occupancy x CUs, so every workgroup is placed at
  // once on an otherwise idle device).  Residency is not guaranteed by the launch, and need not be: every spin is
  // bounded, so a grid that is not resident aborts and its unfinished windows go to the grid-wide path
  // (tests/test_gpu_medium.py forces that path).  The cooperative launch (DVH_CHAIN_LAUNCH=coop) guarantees residency
  // but makes the HIP runtime's exit-time teardown fault under rocprofv3 (SIGSEGV in libhsa-runtime64 called from
  // libamdhip64's exit handler, after the profiler's finalisation; profiles/r04a_chain_exit_crash.txt), same speed.
  static const bool coop = [] {
    const char* v = getenv("DVH_CHAIN_LAUNCH");
    return v && strcmp(v, "coop") == 0;
  }();
  if (coop)
    return hipLaunchCooperativeKernel((const void*)pdhg_chain_kernel, dim3(8 * S), dim3(kCB), args, (unsigned)lds, s);
  hipLaunchKernelGGL(pdhg_chain_kernel, dim3(8 * S), dim3(kCB), lds, s, bb, ww, cc, oo, a);
  return hipGetLastError();
}

namespace {
__global__ void chain_mark_kernel(int32_t* istats, const int32_t* list, int nlist) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nlist) istats[2 * (int64_t)list[i]] = kChainPending;
}
}  // namespace

hipError_t launch_chain_mark(const Batch& b, const int32_t* list, int nlist, hipStream_t s) {
  if (nlist <= 0) return hipSuccess;
  hipLaunchKernelGGL(chain_mark_kernel, dim3((nlist + 255) / 256), dim3(256), 0, s, b.istats, list, nlist);
  return hipGetLastError();
}

hipError_t launch_setup_long(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int k, const int64_t* d,
                             hipStream_t s) {
  LongArgs a;
  a.b = b;
  a.w = w;
  a.k = k;
  a.kl = k - ch.first;
  a.n = (int)d[0];
  a.m = (int)d[1];
  a.T = (int)d[2] - 1;
  a.J = a.n - 3 * a.T;
  a.W.n = a.n;
  a.W.m = a.m;
  a.W.meq = (int)d[2];
  a.W.nnz = (int)d[3];
  a.W.row = d[4];
  a.W.nz = d[5];
  a.W.on = d[6];
  a.W.om = d[7];
  a.W.wn = a.W.on - ch.base_n;
  a.W.wm = a.W.om - ch.base_m;
  a.W.wz = a.W.nz - ch.base_nz;
  a.W.wtr = a.W.wn + a.kl;
  if (a.T < 1 || a.J < 0) return hipErrorInvalidValue;
  const int nb = (std::max(a.n, a.m) + kLB - 1) / kLB;
  if (4 * (int64_t)nb > a.m) return hipErrorInvalidValue;  // norm partials in the window's wbuf
  hipLaunchKernelGGL(long_init, dim3(nb), dim3(kLB), 0, s, a);
  for (int pass = 0; pass <= o.ruiz_iters; ++pass) {
    const bool pc = pass == o.ruiz_iters;
    if (pc) {
      hipLaunchKernelGGL(long_pass<false>, dim3(nb), dim3(kLB), 0, s, a);
      if (a.J) hipLaunchKernelGGL(long_tau_pass<false>, dim3(a.J), dim3(kLB), 0, s, a);
    } else {
      hipLaunchKernelGGL(long_pass<true>, dim3(nb), dim3(kLB), 0, s, a);
      if (a.J) hipLaunchKernelGGL(long_tau_pass<true>, dim3(a.J), dim3(kLB), 0, s, a);
    }
    hipLaunchKernelGGL(long_apply, dim3(nb), dim3(kLB), 0, s, a);
  }
  hipLaunchKernelGGL(long_fill, dim3(nb), dim3(kLB), 0, s, a);
  hipLaunchKernelGGL(long_norms, dim3(1), dim3(kLB), 0, s, a, nb, o.step_safety);
  return hipGetLastError();
}

}  // namespace dvh

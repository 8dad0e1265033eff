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
// Mapping: B lanes per window, lane l owns the S consecutive time steps S l .. S l + S - 1 -- their columns, their
// SOE / DCM (/ ICE) rows -- with every coefficient, bound, objective, iterate and anchor in VGPRs.  An SpMV needs
// only the next step's ene (K x) and the previous SOE row's dual (K^T y); inside a lane those are registers, across
// lanes one LDS store + one LDS load per lane and half-step.  The dense tau columns are summed by wave 0 from
// per-lane partials.  Instantiations: <768, 1> (one step per lane, 12 waves, one window per CU) and <384, 2> (two
// steps per lane, 6 waves: two windows share a CU, so one window's barrier waits are filled by the other's work,
// and every lane carries two independent FMA chains).  <= 168 VGPRs (3 waves per SIMD) either way.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "dvh_device.h"

namespace dvh {
namespace {

constexpr int kBandSteps = 768;  // steps per window (T <= kBandSteps)
constexpr int kJMax = 4;         // tau (demand-period) columns per window
constexpr int kNeedsEll = -2;

// LDS layout (B lanes, S steps per lane, SB = S B steps), doubles then ints:
//   XE[B+1] YS[B+1] XT[kJMax] red[kNRed(NW+1)+4] TP[kJMax][B] XP[NC S][B] YP[NR S][B] (ICE: RO[6 S][B])
//   | ints: dcm[SB] ice_a[SB] ice_b[SB] ice_n[SB] flag[4]
// Register-relief flags LF (forms with several steps per lane): kLfAnchors -- the Halpern anchors XA[NC S][B] /
// YA[NR S][B] live in LDS (one FMA operand per iteration, written at restarts; the ints, read only while the lane
// state is loaded, share their space); kLfCosts -- CQ[5 S][B] = c of ch / dis / ene and q of the SOE / DCM rows in
// LDS (one FMA addend per iteration); kLfImages -- the check iteration's T(z_k) goes to the window's global workspace
// instead of XP / YP (read back by the same lane at the check).  Layout after TP: [XP YP] (no kLfImages) [XA YA]
// (kLfAnchors) [RO] (ICE) [CQ] (kLfCosts).
constexpr int kLfAnchors = 1, kLfCosts = 2, kLfImages = 4;
#ifndef DVH_BAND_TAU_WAVESUMS
#define DVH_BAND_TAU_WAVESUMS 0
#endif
// tau_parts (below): per-wave sums of one tau column.  Off: the same-box bench A/B found no difference (227.5k vs
// 227.7k windows/s, profiles/r04g_ab_band_tau_wavesums.log); the round-3 arithmetic (certified) is kept.
constexpr bool kTauWaveSums = DVH_BAND_TAU_WAVESUMS != 0;
// Where the band iteration's time goes (round 5): wave 0 reduces and updates the single tau column of a monthly window
// (J = 1) at the start of the primal half-step, and the other waves wait for it at the first barrier -- per wave
// (scripts/probe_band_latency.py, profiles/r05b_band_latency.log) wave 0's primal half-step takes 996-1024 shader cycles
// against 610-640 for the others, who wait 390-440 cycles there.  Measured and not kept (profiles/r05c_*, r05g_*): a
// replica of the column in every wave updated in the primal half-step (1.099 vs 1.048 us per window-iteration per
// slot) and the column updated in the dual half-step by every wave (1.146): every wave then carries the chain; the
// costs read from LDS ahead of the second barrier (1.136: the compiler holds them through the iteration).  Ablations at
// a fixed iteration count (wrong results; profiles/r05h_band_ablations.log, r05k_*) bound what is left: without the tau
// chain -7 %, without both barriers -9 %, without the cost / right-hand-side LDS reads -7.5 %, all together -24 %.
__host__ __device__ inline size_t band_lds_doubles(int B, int S, bool ice, int LF) {
  const int NW = B / kWave, NC = ice ? 5 : 3, NR = ice ? 4 : 2;
  const size_t SB = (size_t)S * B;
  return 2 * (size_t)(B + 1) + kJMax + (size_t)kNRed * (NW + 1) + 4 + (size_t)kJMax * B +
         ((LF & kLfImages) ? 0 : (NC + NR) * SB) + ((LF & kLfAnchors) ? (NC + NR) * SB : 0) +
         ((LF & kLfCosts) ? 5 * SB : 0) + (ice ? 6 * SB : 0);
}
__host__ __device__ inline size_t band_ints_bytes(int B, int S) { return sizeof(int32_t) * (4 * (size_t)S * B + 4); }
// The ints share the anchors' (kLfAnchors) or, in the other relieved forms, the check images' space
__host__ __device__ constexpr bool band_ints_shared(int LF) { return (LF & kLfAnchors) || (LF && !(LF & kLfImages)); }
// (round 6) the lane's DCM row indices, drow[S][B], kept in LDS from the set-up to the write-back instead of in VGPRs (held
// across the iteration loop they were among the persistent form's spilled values, and each check's reload of a spilled
// index waited for every global load issued before it)
__host__ __device__ inline size_t band_drow_bytes(int B, int S) { return align16(sizeof(int32_t) * (size_t)S * B); }
__host__ __device__ inline size_t band_lds_bytes(int B, int S, bool ice, int LF) {
  const size_t d = align16(sizeof(double) * band_lds_doubles(B, S, ice, LF));
  return (band_ints_shared(LF) ? d : d + align16(band_ints_bytes(B, S))) + band_drow_bytes(B, S);
}

// KKT pieces of one column / one row (out of line: the KKT check runs every 128 iterations, and inlined it
// would raise the whole kernel's register allocation).  Scale-free where the check compares large terms: the
// objectives' sums c'x, q'y and the bound term l'lam+ + u'lam- are the same in the scaled space (c~ x~ = c x,
// l~ lam~ = (l / d)(d lam) with lam~ = c~ - K~'y~ the scaled reduced cost, d > 0 keeping its sign), so the gap needs
// no factor at all.  Only the residual norms and ||y|| are unscaled, with fd = the factor in single precision
// (Work::fc / fr) and a 1-ulp v_rcp_f32 reciprocal: each term moves by a relative 2e-7 at most, i.e. each norm by a
// relative 2e-7 of itself.  The outputs are unscaled with the exact factors.
// DVH_KKT_INLINE: 1 (default) the KKT helpers below inlined into the battery forms and called out of line from the ICE
// form; 2 inlined everywhere; 0 out of line everywhere (rounds 1-4, so as not to raise the kernel's register
// allocation).  Out of line, every call binds the caller's live registers to the call ABI: inlined, the persistent
// battery form runs 1.5 % faster per iteration with no checks at all and 0.8-1.2 % on the sweep's check schedules
// (profiles/r05s_check_cost_*.log).  The ICE form (168-VGPR budget, already spilling) runs config 5 5.6 % slower with
// them inlined (106.5k vs 112.9k windows/s, identical iterations; profiles/r05za_config5_bisect.log), although a
// fixed-iteration run with checks that never converge had it 9.4 % faster (profiles/r05u_kkt_inline_ice_chain.log).
#ifndef DVH_KKT_INLINE
#define DVH_KKT_INLINE 1
#endif
template <bool ICE>
constexpr bool kkt_inline() { return DVH_KKT_INLINE == 2 || (DVH_KKT_INLINE == 1 && !ICE); }
struct ColKkt {
  double rd2, cx, bt;
};
struct ColKktX : ColKkt {
  double rdx;  // |r_d| |x| of the column, unscaled (the battery forms' objective gate)
};
__device__ __forceinline__ ColKkt col_kkt_i(double kt, double cj, double loj, double hij, double xj, float fd) {
  const double id = (double)__builtin_amdgcn_rcpf(fd);
  const double rs = cj - kt;  // scaled reduced cost
  const bool fl = isfinite(loj), fh = isfinite(hij);
  const double lam = (fl && fh) ? rs : (fl ? fmax(rs, 0.0) : (fh ? fmin(rs, 0.0) : 0.0));
  const double rd = (rs - lam) * id;
  return {rd * rd, cj * xj, (fl ? loj * fmax(lam, 0.0) : 0.0) + (fh ? hij * fmin(lam, 0.0) : 0.0)};
}
__device__ __forceinline__ ColKktX col_kkt_x_i(double kt, double cj, double loj, double hij, double xj, float fd) {
  const double id = (double)__builtin_amdgcn_rcpf(fd);
  const double rs = cj - kt;  // scaled reduced cost
  const bool fl = isfinite(loj), fh = isfinite(hij);
  const double lam = (fl && fh) ? rs : (fl ? fmax(rs, 0.0) : (fh ? fmin(rs, 0.0) : 0.0));
  const double rd = (rs - lam) * id;
  ColKktX r;
  r.rd2 = rd * rd;
  r.cx = cj * xj;
  r.bt = (fl ? loj * fmax(lam, 0.0) : 0.0) + (fh ? hij * fmin(lam, 0.0) : 0.0);
  r.rdx = fabs(rd) * fabs(xj * (double)fd);
  return r;
}
struct RowKkt {
  double rp2, y2;
};
__device__ __forceinline__ RowKkt row_kkt_i(double kv, double qi, double yi, float fd, int ge) {
  const double dr = (double)fd, idr = (double)__builtin_amdgcn_rcpf(fd);
  double r = (qi - kv) * idr;
  if (ge) r = fmax(r, 0.0);
  return {r * r, (yi * dr) * (yi * dr)};
}
__device__ __noinline__ ColKkt col_kkt_o(double kt, double cj, double loj, double hij, double xj, float fd) {
  return col_kkt_i(kt, cj, loj, hij, xj, fd);
}
__device__ __noinline__ ColKktX col_kkt_x_o(double kt, double cj, double loj, double hij, double xj, float fd) {
  return col_kkt_x_i(kt, cj, loj, hij, xj, fd);
}
__device__ __noinline__ RowKkt row_kkt_o(double kv, double qi, double yi, float fd, int ge) {
  return row_kkt_i(kv, qi, yi, fd, ge);
}
template <bool INL>
__device__ __forceinline__ ColKkt col_kkt_fn(double kt, double cj, double loj, double hij, double xj, float fd) {
  if constexpr (INL) return col_kkt_i(kt, cj, loj, hij, xj, fd);
  else return col_kkt_o(kt, cj, loj, hij, xj, fd);
}
template <bool INL>
__device__ __forceinline__ ColKktX col_kkt_fn_x(double kt, double cj, double loj, double hij, double xj, float fd) {
  if constexpr (INL) return col_kkt_x_i(kt, cj, loj, hij, xj, fd);
  else return col_kkt_x_o(kt, cj, loj, hij, xj, fd);
}
template <bool INL>
__device__ __forceinline__ RowKkt row_kkt_fn(double kv, double qi, double yi, float fd, int ge) {
  if constexpr (INL) return row_kkt_i(kv, qi, yi, fd, ge);
  else return row_kkt_o(kv, qi, yi, fd, ge);
}

// GATE: the predicted KKT gate (dvh_options.kkt_predict > 0) is compiled in only where the host asks for it -- its
// state and extra reduction raised the register allocation of the check path by 30-40 spilled VGPRs in every form
// (profiles/r02zzk_ab_configs12_spills.log), which runs with the default options paid for nothing.
//
// BOX (box form, the default): every ch / dis / ene (/ elec / on) column has a finite box [lo, hi] in the
// scaled space, so the kernel iterates on x' = (x - lo) / w, w = hi - lo, whose box is [0, 1]: the projection is the
// FMA's own clamp modifier (one v_fma_f64 ... clamp instead of v_fma + v_max + v_min per column and iteration).  The
// change of variables is exact: K' = K diag(w) (both SpMV directions), c' = c w, q' = q - K lo, and a per-column
// primal step tau / w^2 gives x' + (tau / w^2)(w g) = (x + tau g - lo) / w, i.e. the same PDHG iterates.  The
// movement norms that drive restarts and the primal weight are taken in x units (w d'), the KKT check runs on the
// primed LP, whose objectives, row residuals and (zero, for a two-sided box) column residuals equal the original's
// once the constant c lo is added.  A window with an unbounded ch / dis / ene (/ elec / on) column is returned with
// status kNeedsPlain and re-run by the plain form (dvh_api.cpp device_cascade).
constexpr int kNeedsPlain = -3;
// kBoxRescale (box form): the checks and restarts stop re-reading the columns' box widths from the window's workspace
// in HBM.  A restart rescales the per-column steps tau / w^2 by tau_new / tau_old (one uniform quotient, no per-column
// division), and the check iteration's movement norms, in x units, weigh each column's d'^2 by w^2 = tau / step (an
// approximate reciprocal: the norms only steer restarts and the primal weight).  Before, each check iteration loaded
// the 9 widths of its three steps and each restart loaded them again and divided 9 times.
#ifndef DVH_BAND_RSTEP
#define DVH_BAND_RSTEP 1
#endif
constexpr bool kBoxRescale = DVH_BAND_RSTEP != 0;
// kNoWidths (round 6, box form): the columns' widths are not kept in the window's workspace -- the steps are formed
// from the registers at set-up, the restarts rescale them (kBoxRescale), and the write-back recomputes w = u / d - l / d
// with the operations of the set-up (bit-identical): one write and one read of 8 bytes per column less per window.
#ifndef DVH_BAND_NOWIDTHS
#define DVH_BAND_NOWIDTHS 1
#endif
constexpr bool kNoWidths = kBoxRescale && DVH_BAND_NOWIDTHS != 0;
// DVH_BAND_F32F (A/B, off): the Ruiz / Pock-Chambolle factors rounded to single precision once, when the scaling passes
// end (1: the outputs unscaled from the single-precision copy, which is then the factor exactly, and the factors no
// longer written in double; -1: rounded only).  Measured and not kept (profiles/r06b_t2_rounded_factors.log): the
// degenerate two-step window of tests/test_gpu_configs.py::test_band_kernel_forms_agree[2] (two demand periods of one
// step each) converges in 10,496 / 3,968 iterations (three-step / one-step form) with the exact factors and not at all
// (20,000) with the rounded ones -- a 1e-8 change of the preconditioner moves PDHG's path on that window that much.
#ifndef DVH_BAND_F32F
#define DVH_BAND_F32F 0
#endif
constexpr bool kF32Factors = DVH_BAND_F32F > 0;
constexpr bool kF32Round = kF32Factors || DVH_BAND_F32F == -1;
// kHalpernDiv (round 6): the 64 Halpern weights 1 / (k + 2) of the next block of iterations are divided in the lanes
// (one correctly rounded quotient per lane: the table's values, bit for bit) instead of loaded from the global table.
// The load sat on the restart path: a restart resets k to 0 and the very next iteration reads weight 0, so every
// restart waited for a global load (and the table pointer was one of the values the persistent loop spilled).
#ifndef DVH_BAND_HDIV
#define DVH_BAND_HDIV 1
#endif
constexpr bool kHalpernDiv = DVH_BAND_HDIV != 0;
// kkt_prefetch (round 6): a KKT check reads the single-precision factors of the lane's columns and rows (Work::fc / fr,
// 15 per lane) from the window's workspace.  Each load sat behind its opaque index (kept so that the check's address
// arithmetic is not hoisted into the iteration loop) and was waited for before the next one was issued: 15 serialised
// global-memory latencies per check (the ISA showed each global_load_dword followed by s_waitcnt vmcnt(0)).  Now the
// indices and loads are issued together at the top of the check, one wait behind the image reads and the barrier.
#ifndef DVH_BAND_KKT_PREFETCH
#define DVH_BAND_KKT_PREFETCH 1
#endif
// (the ICE form, at its 168-VGPR budget, spills 14 VGPRs more with the batched loads and runs config 5 slower: 111.9k vs
// 114.7k windows/s, profiles/r06c_ab.log -- it keeps the per-use loads)
#ifndef DVH_BAND_KKT_PREFETCH_ICE
#define DVH_BAND_KKT_PREFETCH_ICE 0
#endif
template <bool ICE>
constexpr bool kkt_prefetch() { return DVH_BAND_KKT_PREFETCH != 0 && (!ICE || DVH_BAND_KKT_PREFETCH_ICE != 0); }
// DVH_BAND_PRIO (round 6, default 2): wave 0, whose primal half-step carries the tau column's reduction and update --
// the iteration's critical path, on which the other three waves wait at the first barrier -- raises its issue priority
// (s_setprio) until that barrier, so that the SIMD it shares with the other window's wave issues its instructions
// first.  Measured (scripts/gpu_r06a.sh, profiles/r06a_ab.log): 0.979 -> 0.940 us per window-iteration per slot at a
// fixed 1,024 iterations, bench 284.4k -> 292.9k windows/s, identical iterations and residuals; config 5 (the ICE form,
// whose wave 0 of twelve carries the column) 108.3k -> 111.9k (profiles/r06c_ab.log).  0: off.
#ifndef DVH_BAND_PRIO
#define DVH_BAND_PRIO 2
#endif
// (DVH_BAND_PRIO_SETUP, A/B, off) the same for the set-up's tau reductions on wave 0 (every scaling pass and power-iteration
// step): measured slower, 290.2k vs 292.3k windows/s (profiles/r06i_prio_setup.log) -- there the raised wave takes issue
// slots from the other window's iterations
#ifndef DVH_BAND_PRIO_SETUP
#define DVH_BAND_PRIO_SETUP 0
#endif
constexpr bool kPrioSetup = DVH_BAND_PRIO_SETUP != 0;
// DVH_BAND_PRIO_DUAL (A/B): every wave raises its priority from the start of the dual half-step until its DCM rows'
// tau partials are written (the values wave 0's next reduction waits for).  Measured and not kept: 292.0k vs 292.6k
// windows/s (profiles/r06c_ab.log); s_setprio 3 instead of 2 for wave 0: 292.7k (same).
// DVH_BAND_PIN_BLEND (A/B): wave 0 finishes the iteration's Halpern blends (x = ca x-bar + cb x-anchor, and the rows')
// before the second barrier, where it waits for the others anyway, instead of after it: the compiler sank them past the
// barrier, to the head of wave 0's next primal half-step -- in front of the tau reduction, at normal priority.
// Measured (profiles/r06j_pin_blend.log): bench 293.1k -> 298.1k windows/s, 0.939 -> 0.930 us per window-iteration per
// slot at a fixed 1,024 iterations, identical iterations and residuals.
#ifndef DVH_BAND_PIN_BLEND
#define DVH_BAND_PIN_BLEND 1
#endif
// DVH_BAND_LATE_SOE: the waves without the tau column update the SOE rows of their lanes' steps 0 .. S - 2 after the
// second barrier instead of before it (those duals are read only by the lane's own next primal half-step), so that they
// reach the barrier -- which wave 0's next tau reduction waits behind -- sooner.  With 15 spilled VGPRs it was within the
// bench's spread (298.7k vs 297.9k, profiles/r06k_late_soe.log); with the spills gone (DVH_BAND_UWIN) bench 300.1k ->
// 304.6k windows/s, config 5 unchanged (profiles/r06s_ab.log).
// DVH_BAND_PIN_KX (A/B): the waves without the tau column finish their primal half-step's own-column K x-bar (x-bar =
// 2 p - x, then K x-bar - q of their rows) before the first barrier, where they wait for wave 0 anyway, instead of after
// it: the compiler sank that work into their dual half-step, which is the critical path into the second barrier.
// Measured (profiles/r06l_pin_kx.log): config 5 (the ICE form: eleven such waves) 116.5k -> 126.0k windows/s; the bench
// 298.2k -> 298.6k, within its spread, at 25 instead of 15 spilled VGPRs.  1 (default): the ICE form only; 2: every form.
#ifndef DVH_BAND_PIN_KX
#define DVH_BAND_PIN_KX 1
#endif
// DVH_BAND_LATE_ICE: the same waves update the two ICE rows' duals (read only by the lane's own next primal
// half-step) after the second barrier instead of before it.  Measured (profiles/r06m_late_ice.log): config 5
// 126.0k -> 127.9-128.4k windows/s.
#ifndef DVH_BAND_LATE_ICE
#define DVH_BAND_LATE_ICE 1
#endif
#ifndef DVH_BAND_LATE_SOE
#define DVH_BAND_LATE_SOE 1
#endif
#ifndef DVH_BAND_PRIO_DUAL
#define DVH_BAND_PRIO_DUAL 0
#endif
// DVH_BAND_PROBE (A/B builds only, scripts/probe_band_latency.py): every wave accumulates the shader-clock cycles of
// its iterations' four segments -- primal half-step, wait at the first barrier, dual half-step, wait at the second --
// and of the checks, and lane 0 writes them over x[6 wid .. 6 wid + 4] of its window at the end, with the wave's
// HW_ID register (SIMD, CU, SE, workgroup slot) in x[6 wid + 5].
#ifndef DVH_BAND_PROBE
#define DVH_BAND_PROBE 0
#endif
__device__ __forceinline__ unsigned long long probe_clock() {
#if DVH_BAND_PROBE
  return __builtin_amdgcn_s_memtime();
#else
  return 0ull;
#endif
}
__device__ __forceinline__ double fma_clamp01(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3 clamp" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// DVH_BAND_UWIN: the window index and its descriptor's offsets are read through v_readfirstlane, so that they and every
// address formed from them (the window's CSR, costs, bounds, outputs, workspace) are scalar.  Loaded as they are -- with
// vector loads, since the kernel writes global memory the compiler does not treat the descriptors as constant -- they sat
// in VGPR pairs, and the base addresses the set-up and the write-back use were spilled.
#ifndef DVH_BAND_UWIN
#define DVH_BAND_UWIN 1
#endif
// DVH_BAND_USCAL: the check path's wave-uniform doubles (the fixed-point residual and the restart test's r0 / rprev, the
// KKT objectives and ratios, the gate's state) through v_readfirstlane, and the residuals' denominators formed where they
// are used: held in SGPR pairs between checks instead of VGPR pairs.  1 (default): the ICE form only -- at its 168-VGPR
// budget spilled VGPRs 41 -> 19, config 5 +1.3 %; in the battery form (spills 2 -> 0) the bench ran 1.8 % slower
// (profiles/r06r_uscal.log); 2: every form.
#ifndef DVH_BAND_USCAL
#define DVH_BAND_USCAL 1
#endif
template <bool ICE>
__device__ __forceinline__ double usc(double v) {
  return (DVH_BAND_USCAL > 1 || (DVH_BAND_USCAL == 1 && ICE)) ? uniform(v) : v;
}
// a uniform double the optimiser must re-read where it is used (so that what is formed from it is not hoisted out of the
// iteration loop into a long-lived VGPR pair)
template <bool ICE>
__device__ __forceinline__ double sgpr_fresh(double v) {
  if constexpr (DVH_BAND_USCAL > 1 || (DVH_BAND_USCAL == 1 && ICE)) asm volatile("" : "+s"(v));
  return v;
}
template <int B, int S, bool ICE, int LF, int WPS, bool GATE, bool BOX>
__device__ __forceinline__ void band_window(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, const int k_in,
                                            const int tid) {
  const int k = DVH_BAND_UWIN ? __builtin_amdgcn_readfirstlane(k_in) : k_in;
  static_assert(!BOX || !(LF & kLfImages), "the box form keeps the check images in LDS");
  constexpr int NW = B / kWave;
  constexpr int SB = S * B;        // step capacity
  constexpr int NC = ICE ? 5 : 3;  // columns per step: ch, dis, ene (, elec, on)
  constexpr int NR = ICE ? 4 : 2;  // rows per step: SOE, DCM (, ICE rated, ICE minimum)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int kl = k - ch.first;
  const WinOff W = DVH_BAND_UWIN ? uniform_win(win_offsets(b, ch, k)) : win_offsets(b, ch, k);
  const int n = W.n, m = W.m, meq = W.meq;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* scal = w.scal + (int64_t)kl * kScal;
  const int T = meq - 1, J = n - (ICE ? 5 : 3) * T, MI = m - meq;
  const int MD = ICE ? MI - 2 * T : MI;  // DCM rows
  auto bail = [&]() {
    if (tid == 0) {
      b.istats[2 * k] = kNeedsEll;
      b.istats[2 * k + 1] = 0;
    }
  };
  // the kernel scales its windows itself (below): it runs before, and instead of, setup_kernel, whose outputs it
  // does not read; the windows it hands on are set up after it (dvh_api.cpp device_cascade)
  if (n > kSmallMax || m > kSmallMax || T < 1 || T > SB || J < 0 || J > kJMax || MD < 0 || MD > T ||
      (J == 0 && MD > 0)) {
    bail();
    return;
  }
  const int CE = 3 * T + J, CO = 4 * T + J;  // first elec / on column (ICE)
  // ---- LDS carve
  double* XE = reinterpret_cast<double*>(smem);  // x-bar (x+) of ene of lane l's first step at [l]; [B] stays 0
  double* YS = XE + (B + 1);  // y (y+) of the init row at [0], of the SOE row of lane l's last step at [l + 1]
  double* XT = YS + (B + 1);  // x-bar (x+) of the tau columns
  double* red = XT + kJMax;
  double* TP = red + kNRed * (NW + 1) + 4;  // [kJMax][B] per-lane partial K'y of the tau columns
  constexpr bool LA = LF & kLfAnchors, LC = LF & kLfCosts, LI = LF & kLfImages;
  double* XP = TP + kJMax * B;                  // [NC S][B] T(z) of the lane's columns (check iterations)
  double* YP = XP + (LI ? 0 : NC * SB);         // [NR S][B] T(z) of the lane's rows
  double* XA = YP + (LI ? 0 : NR * SB);         // [NC S][B] Halpern anchors of the columns (kLfAnchors)
  double* YA = XA + (LA ? NC * SB : 0);         // [NR S][B] and of the rows
  // ICE: read-only data of the ICE columns / rows in LDS instead of VGPRs (the register budget at 3 waves per
  // SIMD is 168): RO[0..1] = c of elec / on, RO[2..3] = upper bound of elec / on, RO[4..5] = q of the two ICE rows,
  // each [S][B]
  double* RO = YA + (LA ? NR * SB : 0);
  double* CQ = RO + (ICE ? 6 * SB : 0);  // [5 S][B] (kLfCosts)
  static_assert(!LA || sizeof(double) * (NC + NR) * SB >= sizeof(int32_t) * (4 * SB + 4), "ints fit the anchors");
  constexpr bool IS = band_ints_shared(LF);  // the ints share the anchors' / images' LDS
  int32_t* dcm = LA   ? reinterpret_cast<int32_t*>(XA)
                 : IS ? reinterpret_cast<int32_t*>(XP)
                      : reinterpret_cast<int32_t*>(smem + align16(sizeof(double) * band_lds_doubles(B, S, ICE, LF)));
  int32_t* ice_a = dcm + SB;  // [SB] ICE rows of each step (lower / higher row index), and their count
  int32_t* ice_b = ice_a + SB;
  int32_t* ice_n = ice_b + SB;
  int32_t* flag = ice_n + SB;
  int32_t* DRL = reinterpret_cast<int32_t*>(smem + band_lds_bytes(B, S, ICE, LF) - band_drow_bytes(B, S));  // [S][B]

  const int32_t* gkp = b.indptr + W.row;
  const int32_t* gkc = b.indices + W.nz;
  const double* gkv = b.data + W.nz;  // the window's own (unscaled) data
  const double* craw = b.c + W.on;
  const double* lraw = b.l + W.on;
  const double* uraw = b.u + W.on;
  const double* qraw = b.q + W.om;
  double* dcv = w.dc + W.wn;  // the factors this kernel computes (outputs are unscaled with them; !kF32Factors)
  double* drv = w.dr + W.wm;
  // the factor of column j / row i at the write-back: the single-precision copy is the factor itself (kF32Factors)
  auto dcf = [&](int j) -> double { return kF32Factors ? (double)w.fc[W.wn + j] : dcv[j]; };
  auto drf = [&](int i) -> double { return kF32Factors ? (double)w.fr[W.wm + i] : drv[i]; };
  double* xo_g = b.x + W.on;
  double* yo_g = b.y + W.om;

  // ---- structure check (every entry of every row accounted for) and the step -> row maps
  for (int u = tid; u < SB; u += B) {
    dcm[u] = -1;
    ice_a[u] = 0x7fffffff;
    ice_b[u] = -1;
    ice_n[u] = 0;
  }
  if (tid == 0) flag[0] = flag[1] = flag[2] = 0;
  __syncthreads();
  int bad = 0, crossed = 0, unboxed = 0;
  for (int j = tid; j < J; j += B) crossed |= lraw[3 * T + j] > uraw[3 * T + j];
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
    // the kernel keeps no lower bound for ch / dis (/ elec / on); crossed bounds: infeasible as given
    bad |= lraw[t] != 0.0 || lraw[T + t] != 0.0;
    crossed |= lraw[t] > uraw[t] || lraw[T + t] > uraw[T + t] || lraw[2 * T + t] > uraw[2 * T + t];
    if (BOX) unboxed |= !(isfinite(uraw[t]) && isfinite(uraw[T + t]) && isfinite(lraw[2 * T + t]) && isfinite(uraw[2 * T + t]));
    if (ICE) {
      if (BOX) unboxed |= !(isfinite(uraw[CE + t]) && isfinite(uraw[CO + t]));
      bad |= lraw[CE + t] != 0.0 || lraw[CO + t] != 0.0;
      crossed |= lraw[CE + t] > uraw[CE + t] || lraw[CO + t] > uraw[CO + t];
    }
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
  if (crossed) flag[1] = 1;
  if (unboxed) flag[2] = 1;
  __syncthreads();
  if (ICE)
    for (int u = tid; u < T; u += B)
      if (ice_n[u] != 2) flag[0] = 1;  // exactly two ICE rows per step
  __syncthreads();
  if (flag[1] != 0) {  // crossed bounds, reported as setup_kernel reports them (no iterations)
    if (tid == 0) {
      scal[0] = 0.0;
      scal[6] = 3.0;
      b.istats[2 * k] = 1;  // DVH_PRIMAL_INFEASIBLE
      b.istats[2 * k + 1] = 0;
      for (int u = 0; u < 4; ++u) b.stats[4 * k + u] = u == 0 ? NAN : 0.0;
    }
    return;
  }
  if (flag[0] != 0) {
    bail();
    return;
  }
  auto bail_plain = [&]() {
    if (tid == 0) {
      b.istats[2 * k] = kNeedsPlain;
      b.istats[2 * k + 1] = 0;
    }
  };
  if (BOX && flag[2] != 0) {
    bail_plain();
    return;
  }

  // ---- the lane's steps t = S tid + s: columns (v) ch, dis, ene (, elec, on), rows (r) SOE, DCM (, ICE a, ICE b)
  const int t0 = S * tid;
  bool val[S];
  double x[S][NC], xa[S][NC], cc[S][3], hi[S][3];
  double loe[S];                     // lower bound of ene (the others are 0)
  double ks[S][4];                   // SOE row: coefficients of ch_t, dis_t, ene_t, ene_{t+1}
  double kd[S][4];                   // DCM row: coefficients of ch_t, dis_t, tau_j, elec_t
  double ka[S][2], kb[S][2];         // ICE rows: coefficients of elec_t, on_t
  double kp0 = 0.0;                  // coefficient of ene_{t0} in row t0 (the init row or the previous lane's SOE
                                     // row); for s > 0 the coefficient of ene_t in row t is ks[s - 1][3]
  double y[S][NR], ya[S][NR], q[S][2];
  int drow[S], jt[S], ra[S], rb[S];
  auto col = [&](int s, int v) { return v < 3 ? v * T + t0 + s : (v == 3 ? CE : CO) + t0 + s; };
  auto ro = [&](int u, int s) -> double& { return RO[(u * S + s) * B + tid]; };
  auto cqa = [&](int u, int s) -> double& { return CQ[(u * S + s) * B + tid]; };
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int t = t0 + s;
    val[s] = t < T;
#pragma unroll
    for (int v = 0; v < NC; ++v) x[s][v] = xa[s][v] = 0.0;
#pragma unroll
    for (int v = 0; v < 3; ++v) cc[s][v] = hi[s][v] = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r) y[s][r] = ya[s][r] = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) ks[s][u] = kd[s][u] = 0.0;
    ka[s][0] = ka[s][1] = kb[s][0] = kb[s][1] = 0.0;
    q[s][0] = q[s][1] = 0.0;
    loe[s] = 0.0;
    drow[s] = -1;
    DRL[s * B + tid] = -1;
    jt[s] = 0;
    ra[s] = rb[s] = -1;
    if (ICE)
      for (int u = 0; u < 6; ++u) ro(u, s) = 0.0;
    if (LC)
      for (int u = 0; u < 5; ++u) cqa(u, s) = 0.0;
  }
  auto cof = [&](int s, int v) -> double { return v < 3 ? (LC ? cqa(v, s) : cc[s][v]) : ro(v - 3, s); };
  auto qv = [&](int s, int r) -> double { return LC ? cqa(3 + r, s) : q[s][r]; };
  auto hib = [&](int s, int v) -> double { return v < 3 ? hi[s][v] : ro(v - 1, s); };
  auto rhs = [&](int s, int r) -> double { return r < 2 ? qv(s, r) : ro(r + 2, s); };
  // ---- the lane's coefficients (unscaled) and row maps
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (!val[s]) continue;
    const int t = t0 + s;
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
        if (gkc[p] == 2 * T + t) kp0 = gkv[p];
    const int dv = dcm[t];
    if (dv >= 0) {
      drow[s] = dv >> 3;
      DRL[s * B + tid] = drow[s];
      jt[s] = dv & 7;
      for (int p = gkp[drow[s]]; p < gkp[drow[s] + 1]; ++p) {
        const int c = gkc[p];
        const double a = gkv[p];
        if (c < T) kd[s][0] = a;
        else if (c < 2 * T) kd[s][1] = a;
        else if (c < 3 * T + J) kd[s][2] = a;
        else kd[s][3] = a;
      }
    }
    if (ICE) {
      ra[s] = ice_a[t];
      rb[s] = ice_b[t];
      for (int p = gkp[ra[s]]; p < gkp[ra[s] + 1]; ++p) (gkc[p] < CO ? ka[s][0] : ka[s][1]) = gkv[p];
      for (int p = gkp[rb[s]]; p < gkp[rb[s] + 1]; ++p) (gkc[p] < CO ? kb[s][0] : kb[s][1]) = gkv[p];
    }
  }
  // row of step s's r-th row (SOE, DCM, ICE a, ICE b), or -1 where the step has none
  auto row_of = [&](int s, int r) -> int {
    return r == 0 ? (val[s] ? t0 + s + 1 : -1) : r == 1 ? drow[s] : (val[s] ? (r == 2 ? ra[s] : rb[s]) : -1);
  };
  // Special state in wave 0 (registers sp[], meaning by lane): lane j < J holds tau column j {x, xa, c, lo, hi, x+};
  // lane kInitLane holds the init row (row 0: ene_0 = target) {y, ya, y+, q, coefficient, -}.
  constexpr int kInitLane = kWave - 1;
  static_assert(kJMax < kInitLane, "tau lanes and the init-row lane are distinct");
  const bool tlane = wid == 0 && lane < J, ilane = wid == 0 && lane == kInitLane;
  double sp[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};

  // ---- scaling: setup_kernel's preconditioning (o.ruiz_iters Ruiz inf-norm passes, then one Pock-Chambolle
  //      alpha = 1 pass, row and column factors of a pass both from the same scaled matrix) restated on the band
  //      structure, every factor in the registers of the lane that owns the row / column: a row's entries are its
  //      step's columns (+ the next step's ene: the next lane's, through XE; + its period's tau: XT), a column's
  //      entries its step's rows (+ ene's previous SOE row: the previous lane's, through YS); the tau columns are
  //      reduced through TP by wave 0, whose lane j holds tau j's factor (fsp), as lane kInitLane holds the init row's.
  //      Factors 1 / sqrt(norm) by v_rsq_f64: a preconditioner needs no correctly rounded factor, and every scaled
  //      quantity is formed from the same stored factor that unscales the results.
  double fcv[S][NC], frv[S][NR], fsp = 1.0, kin0 = 0.0;  // kin0: the init row's coefficient (of ene_0)
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int v = 0; v < NC; ++v) fcv[s][v] = 1.0;
#pragma unroll
    for (int r = 0; r < NR; ++r) frv[s][r] = 1.0;
  }
  if (ilane) kin0 = gkv[gkp[0]];
  auto factor = [](double a) { return a > 0.0 ? __builtin_amdgcn_rsq(a) : 1.0; };
  auto exchange = [&]() {
    XE[tid] = fcv[0][2];
    YS[tid + 1] = frv[S - 1][0];
    if (tid == 0) XE[B] = 1.0;  // (no step after the last lane's: its coefficient is 0)
    if (tid < kJMax) XT[tid] = tlane ? fsp : 1.0;
    if (ilane) YS[0] = fsp;
  };
  for (int pass = 0; pass <= o.ruiz_iters; ++pass) {
    const bool pc = pass == o.ruiz_iters;
    auto acc = [pc](double a, double v) { return pc ? a + v : fmax(a, v); };
    exchange();
    __syncthreads();
    const double fen = XE[tid + 1], frp = YS[tid];
    double nr[S][NR], nc[S][NC];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double fe1 = s < S - 1 ? fcv[s < S - 1 ? s + 1 : s][2] : fen;
      const double rp = s == 0 ? frp : frv[s > 0 ? s - 1 : 0][0];
      const double kpr = s == 0 ? kp0 : ks[s > 0 ? s - 1 : 0][3];
      const double r0 = frv[s][0], r1 = frv[s][1], ftj = XT[jt[s]];
      nr[s][0] = acc(acc(acc(fabs(ks[s][0]) * r0 * fcv[s][0], fabs(ks[s][1]) * r0 * fcv[s][1]),
                         fabs(ks[s][2]) * r0 * fcv[s][2]),
                     fabs(ks[s][3]) * r0 * fe1);
      nr[s][1] = acc(acc(fabs(kd[s][0]) * r1 * fcv[s][0], fabs(kd[s][1]) * r1 * fcv[s][1]), fabs(kd[s][2]) * r1 * ftj);
      nc[s][0] = acc(fabs(ks[s][0]) * r0 * fcv[s][0], fabs(kd[s][0]) * r1 * fcv[s][0]);
      nc[s][1] = acc(fabs(ks[s][1]) * r0 * fcv[s][1], fabs(kd[s][1]) * r1 * fcv[s][1]);
      nc[s][2] = acc(fabs(kpr) * rp * fcv[s][2], fabs(ks[s][2]) * r0 * fcv[s][2]);
      if constexpr (ICE) {
        const double r2 = frv[s][NR > 2 ? 2 : 0], r3 = frv[s][NR > 3 ? 3 : 0];
        const double f3 = fcv[s][NC > 3 ? 3 : 0], f4 = fcv[s][NC > 4 ? 4 : 0];
        nr[s][1] = acc(nr[s][1], fabs(kd[s][3]) * r1 * f3);
        nr[s][NR > 2 ? 2 : 0] = acc(fabs(ka[s][0]) * r2 * f3, fabs(ka[s][1]) * r2 * f4);
        nr[s][NR > 3 ? 3 : 0] = acc(fabs(kb[s][0]) * r3 * f3, fabs(kb[s][1]) * r3 * f4);
        nc[s][NC > 3 ? 3 : 0] = acc(acc(fabs(kd[s][3]) * r1 * f3, fabs(ka[s][0]) * r2 * f3), fabs(kb[s][0]) * r3 * f3);
        nc[s][NC > 4 ? 4 : 0] = acc(fabs(ka[s][1]) * r2 * f4, fabs(kb[s][1]) * r3 * f4);
      }
    }
    // tau columns: per-lane partials over the lane's DCM rows of each period (steps in order) -> wave 0
    for (int j = 0; j < J; ++j) {
      const double ftj = XT[j];
      double a = 0.0;
#pragma unroll
      for (int s = 0; s < S; ++s)
        if (jt[s] == j) a = acc(a, fabs(kd[s][2]) * frv[s][1] * ftj);
      TP[j * B + tid] = a;
    }
    double nsp = 0.0;
    if (ilane) nsp = fabs(kin0) * fsp * XE[0];
    __syncthreads();
    if (wid == 0) {
      if (DVH_BAND_PRIO && kPrioSetup) __builtin_amdgcn_s_setprio(DVH_BAND_PRIO);
      for (int j = 0; j < J; ++j) {
        double a = TP[j * B + lane];
#pragma unroll
        for (int r = 1; r < NW; ++r) a = acc(a, TP[j * B + r * kWave + lane]);
        a = uniform(pc ? wave_sum_dpp(a) : wave_max(a));
        if (lane == j) nsp = a;
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int v = 0; v < NC; ++v) fcv[s][v] *= factor(nc[s][v]);
#pragma unroll
      for (int r = 0; r < NR; ++r) frv[s][r] *= factor(nr[s][r]);
    }
    if (tlane || ilane) fsp *= factor(nsp);
    __syncthreads();  // every read of this pass's XE / YS / XT / TP is done
    if (DVH_BAND_PRIO && kPrioSetup && wid == 0) __builtin_amdgcn_s_setprio(0);
  }
  {  // the KKT checks unscale with single-precision copies of the factors: a window whose factors leave
     // [2^-100, 2^100] (far inside float's normal range) goes to the ELL / generic path, which keeps them in double
    auto oor = [](double f) { return !(f >= 0x1p-100 && f <= 0x1p100); };
    if constexpr (kF32Round) {  // (round 6) every factor rounded to single precision once, here: the float copy in
                                  // the workspace is then the factor itself, exactly
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int v = 0; v < NC; ++v) fcv[s][v] = (double)(float)fcv[s][v];
#pragma unroll
        for (int r = 0; r < NR; ++r) frv[s][r] = (double)(float)frv[s][r];
      }
      fsp = (double)(float)fsp;
    }
    bool out = oor(fsp);
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int v = 0; v < NC; ++v) out |= oor(fcv[s][v]);
#pragma unroll
      for (int r = 0; r < NR; ++r) out |= oor(frv[s][r]);
    }
    if (__syncthreads_or(out)) {
      bail();
      return;
    }
  }
  exchange();
  __syncthreads();
  {  // scaled coefficients (K Dr) Dc, as setup_kernel forms them
    const double fen = XE[tid + 1], frp = YS[tid];
    kp0 = kp0 * frp * fcv[0][2];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double fe1 = s < S - 1 ? fcv[s < S - 1 ? s + 1 : s][2] : fen;
      const double r0 = frv[s][0], r1 = frv[s][1];
      ks[s][0] = ks[s][0] * r0 * fcv[s][0];
      ks[s][1] = ks[s][1] * r0 * fcv[s][1];
      ks[s][2] = ks[s][2] * r0 * fcv[s][2];
      ks[s][3] = ks[s][3] * r0 * fe1;
      kd[s][0] = kd[s][0] * r1 * fcv[s][0];
      kd[s][1] = kd[s][1] * r1 * fcv[s][1];
      kd[s][2] = kd[s][2] * r1 * XT[jt[s]];
      if constexpr (ICE) {
        const double r2 = frv[s][NR > 2 ? 2 : 0], r3 = frv[s][NR > 3 ? 3 : 0];
        const double f3 = fcv[s][NC > 3 ? 3 : 0], f4 = fcv[s][NC > 4 ? 4 : 0];
        kd[s][3] = kd[s][3] * r1 * f3;
        ka[s][0] = ka[s][0] * r2 * f3;
        ka[s][1] = ka[s][1] * r2 * f4;
        kb[s][0] = kb[s][0] * r3 * f3;
        kb[s][1] = kb[s][1] * r3 * f4;
      }
    }
    if (ilane) kin0 = kin0 * fsp * XE[0];
  }
  // ---- costs, bounds and right-hand sides, scaled (c Dc, l / Dc, u / Dc, q Dr); the factors for the outputs and
  //      the KKT checks; the norms for the primal weight and the relative KKT error
  double nrm[4] = {0.0, 0.0, 0.0, 0.0};  // ||c~||^2, ||q~||^2, ||c||^2, ||q||^2
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (!val[s]) continue;
    const int t = t0 + s;
#pragma unroll
    for (int v = 0; v < NC; ++v) {
      const int j = col(s, v);
      const double d = fcv[s][v], cj = craw[j];
      const double csj = cj * d, lsj = lraw[j] / d, usj = uraw[j] / d;
      if (v < 3) {
        hi[s][v] = usj;
        if (LC)
          cqa(v, s) = csj;
        else
          cc[s][v] = csj;
      } else {
        ro(v - 1, s) = usj;
        ro(v - 3, s) = csj;
      }
      if (v == 2) loe[s] = lsj;
      x[s][v] = xa[s][v] = fmin(fmax(o.warm ? xo_g[j] / d : 0.0, lsj), usj);
      nrm[0] += csj * csj;
      nrm[2] += cj * cj;
      if constexpr (!kF32Factors) dcv[j] = d;
      w.fc[W.wn + j] = (float)d;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int i = row_of(s, r);
      if (i < 0) continue;
      const double d = frv[s][r], qi = qraw[i], qsi = qi * d;
      if (r == 0) {
        if (LC)
          cqa(3, s) = qsi;
        else
          q[s][0] = qsi;
      } else if (r == 1) {
        if (LC)
          cqa(4, s) = qsi;
        else
          q[s][1] = qsi;
      } else {
        ro(r + 2, s) = qsi;
      }
      if (o.warm) y[s][r] = ya[s][r] = r == 0 ? yo_g[i] / d : fmax(yo_g[i] / d, 0.0);
      nrm[1] += qsi * qsi;
      nrm[3] += qi * qi;
      if constexpr (!kF32Factors) drv[i] = d;
      w.fr[W.wm + i] = (float)d;
    }
  }
  if (tlane) {
    const int j = 3 * T + lane;
    const double cj = craw[j], l0 = lraw[j] / fsp, h0 = uraw[j] / fsp;
    sp[0] = sp[1] = sp[5] = fmin(fmax(o.warm ? xo_g[j] / fsp : 0.0, l0), h0);
    sp[2] = cj * fsp;
    sp[3] = l0;
    sp[4] = h0;
    nrm[0] += sp[2] * sp[2];
    nrm[2] += cj * cj;
    if constexpr (!kF32Factors) dcv[j] = fsp;
    w.fc[W.wn + j] = (float)fsp;
  }
  if (ilane) {
    const double q0 = qraw[0];
    sp[3] = q0 * fsp;
    sp[4] = kin0;
    if (o.warm) sp[0] = sp[1] = sp[2] = yo_g[0] / fsp;
    nrm[1] += sp[3] * sp[3];
    nrm[3] += q0 * q0;
    if constexpr (!kF32Factors) drv[0] = fsp;
    w.fr[W.wm] = (float)fsp;
  }
  block_sum<B, 4>(nrm, red);
  const double ncs = sqrt(nrm[0]), nqs = sqrt(nrm[1]);
  const double pw0 = (ncs > 1e-10 && nqs > 1e-10) ? ncs / nqs : 1.0;  // setup_kernel's primal weight
  int xta[S];
#pragma unroll
  for (int s = 0; s < S; ++s) xta[s] = lds_addr(XT + jt[s]);
  if constexpr (IS) __syncthreads();  // anchors / images overwrite the step -> row maps: every lane has read them
  if constexpr (LA) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int v = 0; v < NC; ++v) XA[(v * S + s) * B + tid] = xa[s][v];
#pragma unroll
      for (int r = 0; r < NR; ++r) YA[(r * S + s) * B + tid] = ya[s][r];
    }
  }
  auto axv = [&](int s, int v) -> double { return LA ? XA[(v * S + s) * B + tid] : xa[s][v]; };
  auto ayv = [&](int s, int r) -> double { return LA ? YA[(r * S + s) * B + tid] : ya[s][r]; };
  if (tid < kJMax) XT[tid] = 0.0;
  if (tid == 0) XE[B] = YS[B] = 0.0;
  XE[tid] = YS[tid] = 0.0;
  for (int u = tid; u < kJMax * B; u += B) TP[u] = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (LI) {  // the outputs hold the last KKT check's T(z_k): the starting point until the first one
      if (val[s]) {
#pragma unroll
        for (int v = 0; v < NC; ++v) xo_g[col(s, v)] = x[s][v] * dcf(col(s, v));
      }
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int i = row_of(s, r);
        if (i >= 0) yo_g[i] = y[s][r] * drf(i);
      }
    } else {
#pragma unroll
      for (int v = 0; v < NC; ++v) XP[(v * S + s) * B + tid] = x[s][v];
#pragma unroll
      for (int r = 0; r < NR; ++r) YP[(r * S + s) * B + tid] = y[s][r];
    }
  }
  __syncthreads();

  // ---- SpMV pieces (fixed summation order)
  auto kpv = [&](int s) { return s == 0 ? kp0 : ks[s > 0 ? s - 1 : 0][3]; };
  // K^T of step s's columns from its rows' values vr and vprev = the value of row t (the previous SOE row)
  auto ktr = [&](int s, const double (&vr)[NR], double vprev, double (&out)[NC]) {
    out[0] = fma(kd[s][0], vr[1], ks[s][0] * vr[0]);
    out[1] = fma(kd[s][1], vr[1], ks[s][1] * vr[0]);
    out[2] = fma(ks[s][2], vr[0], kpv(s) * vprev);
    if constexpr (ICE) {
      out[3] = fma(kb[s][0], vr[3], fma(ka[s][0], vr[2], kd[s][3] * vr[1]));
      out[4] = fma(kb[s][1], vr[3], ka[s][1] * vr[2]);
    }
  };
  // K of step s's rows, own-column part (kfin_next adds the next step's ene, kfin_tau the tau term)
  auto kown = [&](int s, const double (&v)[NC], double (&os)[NR]) {
    os[0] = fma(ks[s][2], v[2], fma(ks[s][1], v[1], ks[s][0] * v[0]));
    os[1] = fma(kd[s][1], v[1], kd[s][0] * v[0]);
    if constexpr (ICE) {
      os[1] = fma(kd[s][3], v[3], os[1]);
      os[2] = fma(ka[s][1], v[4], ka[s][0] * v[3]);
      os[3] = fma(kb[s][1], v[4], kb[s][0] * v[3]);
    }
  };
  auto kfin_next = [&](int s, double (&os)[NR], double vnext) { os[0] = fma(ks[s][3], vnext, os[0]); };
  auto kfin_tau = [&](int s, double (&os)[NR]) { os[1] = fma(kd[s][2], lds_ld(xta[s]), os[1]); };
  // The iteration's forms with the objective / right-hand side folded into the FMA chains: K^T y - c for the
  // primal half-step (x + tau (K^T y - c) = x - tau (c - K^T y)) and K x - q for the dual one (y - sigma (K x - q)):
  // one FP64 operation fewer per column and per row than forming the difference afterwards.
  auto ktr_c = [&](int s, const double (&vr)[NR], double vprev, double (&out)[NC]) {
    out[0] = fma(kd[s][0], vr[1], fma(ks[s][0], vr[0], -cof(s, 0)));
    out[1] = fma(kd[s][1], vr[1], fma(ks[s][1], vr[0], -cof(s, 1)));
    out[2] = fma(ks[s][2], vr[0], fma(kpv(s), vprev, -cof(s, 2)));
    if constexpr (ICE) {
      out[3] = fma(kb[s][0], vr[3], fma(ka[s][0], vr[2], fma(kd[s][3], vr[1], -cof(s, 3))));
      out[4] = fma(kb[s][1], vr[3], fma(ka[s][1], vr[2], -cof(s, 4)));
    }
  };
  auto kown_q = [&](int s, const double (&v)[NC], double (&os)[NR]) {
    os[0] = fma(ks[s][2], v[2], fma(ks[s][1], v[1], fma(ks[s][0], v[0], -qv(s, 0))));
    os[1] = fma(kd[s][1], v[1], fma(kd[s][0], v[0], -qv(s, 1)));
    if constexpr (ICE) {
      os[1] = fma(kd[s][3], v[3], os[1]);
      os[2] = fma(ka[s][1], v[4], fma(ka[s][0], v[3], -rhs(s, 2)));
      os[3] = fma(kb[s][1], v[4], fma(kb[s][0], v[3], -rhs(s, 3)));
    }
  };
  // per-lane partial K'y of the tau columns from the DCM rows' values vd[s] (steps summed in order).  One column
  // (J = 1, kTauWaveSums): every wave reduces its lanes' partials itself (one DPP tree, lane 0's sum) into TP[wid],
  // so the tau update on wave 0 adds NW values instead of reducing B partials on the iteration's critical path.
  auto tau_parts = [&](const double (&vd)[S]) {
    if (J == 1) {
      double a = kd[0][2] * vd[0];
#pragma unroll
      for (int s = 1; s < S; ++s) a = fma(kd[s][2], vd[s], a);
      if constexpr (kTauWaveSums) {
        a = wave_sum_dpp(a);
        if (lane == 0) TP[wid] = a;
      } else {
        TP[tid] = a;
      }
    } else {
      for (int j = 0; j < J; ++j) {
        double a = (jt[0] == j ? kd[0][2] : 0.0) * vd[0];
#pragma unroll
        for (int s = 1; s < S; ++s) a = fma(jt[s] == j ? kd[s][2] : 0.0, vd[s], a);
        TP[j * B + tid] = a;
      }
    }
  };
  auto tau_parts_of = [&](const double (&vr)[S][NR]) {
    double vd[S];
#pragma unroll
    for (int s = 0; s < S; ++s) vd[s] = vr[s][1];
    tau_parts(vd);
  };
  // the wave sums of a single tau column, in wave order (every lane reads the same slots: a broadcast)
  auto tau_waves = [&]() {
    double a = TP[0];
#pragma unroll
    for (int r = 1; r < NW; ++r) a += TP[r];
    return a;
  };
  // wave 0: lane j < J gets the sum over all lanes of TP[j][.] (fixed order; uniform per column)
  auto tau_kt = [&]() {
    double res = 0.0;
    if (kTauWaveSums && J == 1) return lane == 0 ? tau_waves() : 0.0;
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
  double eta = o.step_safety;  // Pock-Chambolle bound ||K~|| <= 1, refined by the power iteration
  if (o.power_iters > 0) {
    const int P = o.power_iters;
    const double v0 = 1.0 / sqrt((double)n);
    double vc[S][NC];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int v = 0; v < NC; ++v) vc[s][v] = val[s] ? v0 : 0.0;
    double vtau = (wid == 0 && lane < J) ? v0 : 0.0;
    double nv[2] = {0.0, 0.0};
    double wr[S][NR];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int r = 0; r < NR; ++r) wr[s][r] = 0.0;
    for (int pi = 0; pi <= P; ++pi) {
      // (DVH_BAND_PRIO) wave 0's tau reduction is this step's critical path too, up to the first barrier
      if (DVH_BAND_PRIO && kPrioSetup && wid == 0) __builtin_amdgcn_s_setprio(DVH_BAND_PRIO);
      if (pi > 0) {
        const double ysp = YS[tid];
#pragma unroll
        for (int s = 0; s < S; ++s) ktr(s, wr[s], s == 0 ? ysp : wr[s > 0 ? s - 1 : 0][0], vc[s]);
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
          for (int v = 0; v < NC; ++v) a = fma(vc[s][v], vc[s][v], a);
        nv[pi - (P - 1)] = a;
      }
      if (pi == P) break;
      XE[tid] = vc[0][2];
      if (wid == 0 && lane < J) XT[lane] = vtau;
      __syncthreads();
      if (DVH_BAND_PRIO && kPrioSetup && wid == 0) __builtin_amdgcn_s_setprio(0);
      const double xen = XE[tid + 1];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        kown(s, vc[s], wr[s]);
        kfin_next(s, wr[s], s == S - 1 ? xen : vc[s < S - 1 ? s + 1 : s][2]);
        kfin_tau(s, wr[s]);
      }
      YS[tid + 1] = wr[S - 1][0];
      if (ilane) YS[0] = sp[4] * XE[0];
      tau_parts_of(wr);
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
    YS[tid + 1] = y[S - 1][0];
    if (ilane) YS[0] = sp[0];
    if (J > 0) tau_parts_of(y);
    __syncthreads();
  }
  eta = uniform(eta);
  // A warm start's primal weight: the geometric mean of the data's (||c~|| / ||q~||) and the starting point's own
  // ||y~0|| / ||x~0|| (PDLP's weight is a ratio of dual to primal movement; the start carries the seed's balance).
  // Bench: PDHG 524.5 -> 520.2 ms per step, warm iterations 2,037.5 -> 2,035.5 (profiles/r03q_ab_warm_pw.log); the
  // start's ratio alone: 523.9 ms.
  double pwi = pw0;
  if (o.warm) {
    double nv[2] = {0.0, 0.0};
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int v = 0; v < NC; ++v) nv[0] += x[s][v] * x[s][v];
#pragma unroll
      for (int r = 0; r < NR; ++r) nv[1] += y[s][r] * y[s][r];
    }
    if (tlane) nv[0] += sp[0] * sp[0];
    if (ilane) nv[1] += sp[0] * sp[0];
    block_sum<B, 2>(nv, red);
    if (nv[0] > 1e-20 && nv[1] > 1e-20) {
      const double ratio = sqrt(nv[1] / nv[0]);
      pwi = sqrt(ratio * pw0);
    }
  }
  double pw = uniform(pwi);
  // ---- box form: x' = (x - lo) / w on the ch / dis / ene columns (after the scaling, the power iteration and the
  //      warm start's weight, which all see the original variables)
  double tj[S][3];  // per-column primal steps tau / w^2 of ch / dis / ene (elec / on: in RO, over their upper bounds)
  double* wbox = w.vbuf + W.wn;         // the columns' widths w (window workspace: read at checks, restarts, the end)
  double cbox = 0.0;                    // c lo, the objective's constant under the change of variables
  auto wcol = [&](int s, int v) { return val[s] ? wbox[opaque(col(s, v))] : 0.0; };
  if constexpr (BOX) {
    double wb[S][NC];
    bool unb = false;
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int v = 0; v < NC; ++v) {
        double wv = hib(s, v) - (v == 2 ? loe[s] : 0.0);  // padding steps: 0
        unb |= !isfinite(wv);
        if (!(wv >= 0x1p-500)) wv = 0.0;  // a (numerically) fixed column: x' = 0, x = lo
        wb[s][v] = wv;
      }
    }
    if (__syncthreads_or(unb)) {
      bail_plain();
      return;
    }
    // the next lane's first ene (width, lower bound) for the lane's last SOE row; step 0's for the init row
    XP[tid] = wb[0][2];
    XP[B + 1 + tid] = loe[0];
    if (tid == 0) XP[B] = XP[2 * B + 1] = 0.0;
    __syncthreads();
    const double wnx = XP[tid + 1], lnx = XP[B + 2 + tid], we0 = XP[0], le0 = XP[B + 1];
    __syncthreads();  // (XP is rewritten with the images below)
    double cl[1] = {0.0};
    kp0 *= wb[0][2];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double wn1 = s < S - 1 ? wb[s < S - 1 ? s + 1 : s][2] : wnx;
      const double ln1 = s < S - 1 ? loe[s < S - 1 ? s + 1 : s] : lnx;
      if (val[s]) {  // q' = q - K lo over the SOE row: its ene_t and ene_{t+1} terms (ch / dis have lo = 0)
        const double qs = fma(-ks[s][3], ln1, fma(-ks[s][2], loe[s], qv(s, 0)));
        if (LC)
          cqa(3, s) = qs;
        else
          q[s][0] = qs;
        cl[0] = fma(cof(s, 2), loe[s], cl[0]);
      }
      ks[s][0] *= wb[s][0];
      ks[s][1] *= wb[s][1];
      ks[s][2] *= wb[s][2];
      ks[s][3] *= wn1;
      kd[s][0] *= wb[s][0];
      kd[s][1] *= wb[s][1];
      if constexpr (ICE) {  // elec / on: the DCM row's elec term, the two ICE rows (their q: lo = 0, unchanged)
        const double we = wb[s][NC > 3 ? 3 : 0], wo = wb[s][NC > 4 ? 4 : 0];
        kd[s][3] *= we;
        ka[s][0] *= we;
        ka[s][1] *= wo;
        kb[s][0] *= we;
        kb[s][1] *= wo;
      }
#pragma unroll
      for (int v = 0; v < NC; ++v) {
        const double lo = v == 2 ? loe[s] : 0.0, wv = wb[s][v], cs = cof(s, v) * wv;
        if (v >= 3)
          ro(v - 3, s) = cs;
        else if (LC)
          cqa(v, s) = cs;
        else
          cc[s][v] = cs;
        const double xv = wv > 0.0 ? fmin(fmax((x[s][v] - lo) / wv, 0.0), 1.0) : 0.0;
        x[s][v] = xa[s][v] = xv;
        if constexpr (LA) XA[(v * S + s) * B + tid] = xv;
        XP[(v * S + s) * B + tid] = xv;
        if constexpr (!kNoWidths) {
          if (val[s]) wbox[col(s, v)] = wv;
        } else if (v < 3) {  // the steps tau / w^2 from the registers (box_steps below reads them back otherwise)
          tj[s][v < 3 ? v : 0] = wv > 0.0 ? uniform(eta / pw) / (wv * wv) : 0.0;
        } else {
          ro(v - 1, s) = wv > 0.0 ? uniform(eta / pw) / (wv * wv) : 0.0;
        }
      }
    }
    if (ilane) {
      sp[3] = fma(-sp[4], le0, sp[3]);
      sp[4] *= we0;
    }
    block_sum<B, 1>(cl, red);
    cbox = cl[0];
  }
  const double cnorm = uniform(sqrt(nrm[2])), qnorm = uniform(sqrt(nrm[3])), c0 = uniform(b.c0[k] + cbox);
  int it = 0, kin = 0, status = kIterLimit;
  double r0 = -1.0, rprev = -1.0;
  double* fin = red + kNRed * NW;
  if (tid == 0)
    for (int u = 0; u < 4; ++u) fin[u] = NAN;
  const int chk = o.check_every > 0 ? o.check_every : 64;
  double tau = uniform(eta / pw), sigma = uniform(eta * pw);
  double sigma2n = uniform(-2.0 * sigma);  // the equality rows' fused dual step (non-check iterations)
  double tau_bs = tau;                     // (kBoxRescale) the tau the box steps were last formed for
  auto box_steps = [&]() {
    if constexpr (BOX) {
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int v = 0; v < NC; ++v) {
          const double wv = wcol(s, v), st = wv > 0.0 ? tau / (wv * wv) : 0.0;
          if (v < 3)
            tj[s][v < 3 ? v : 0] = st;
          else
            ro(v - 1, s) = st;
        }
    }
  };
  if constexpr (!kNoWidths) box_steps();  // (kNoWidths: formed at the box set-up)
  // (kBoxRescale) the steps for a new tau from the current ones: tau / w^2 = (tau / tau_bs) (tau_bs / w^2)
  auto box_steps_rescale = [&]() {
    if constexpr (BOX) {
      if constexpr (kBoxRescale) {
        const double f = uniform(tau / tau_bs);
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int v = 0; v < NC; ++v) {
            if (v < 3)
              tj[s][v < 3 ? v : 0] *= f;
            else
              ro(v - 1, s) *= f;
          }
        tau_bs = tau;
      } else {
        box_steps();
      }
    }
  };
  const int kkt_every = o.kkt_every > 0 ? o.kkt_every : 1;
  int ck = chk, kk_ = kkt_every;
  KktGate gate;  // dvh_options.kkt_predict (dvh_device.h)
  int kbase = 0;
  auto hload = [&](int k0_) {
    const int kq = k0_ + lane;
    if constexpr (kHalpernDiv)  // (round 6) no global load on the restart path: the IEEE quotient the table holds
      return 1.0 / (kq + 2.0);
    else
      return kq < kHalpernTab ? w.hinv[kq] : 1.0 / (kq + 2.0);
  };
  double hw = hload(0);

  // wave 0 with one tau column: the tau reduction is interleaved with its own column work (straight-line code,
  // the partial loads are issued first); J >= 2 takes the generic per-column loop
  const bool w0 = wid == 0 && J == 1;
  double mv0, mv1, mv2, mv3;
  double mvb0 = 0.0, mvb1 = 0.0;  // (kBoxRescale) the box columns' movements, d'^2 / step
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
  // Lean form: the check iteration's T(z_k) (scaled) goes to the window's global workspace (the lane reads back only
  // its own entries, at the check); padding steps write nothing
  double* xim = w.vbuf + W.wn;
  double* yim = w.wbuf + W.wm;
  auto load_images = [&](double (&xp)[S][NC], double (&yp)[S][NR]) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if constexpr (LI) {
#pragma unroll
        for (int v = 0; v < NC; ++v) xp[s][v] = val[s] ? xim[opaque(col(s, v))] : 0.0;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int i = row_of(s, r);
          yp[s][r] = i >= 0 ? yim[opaque(i)] : 0.0;
        }
      } else {
#pragma unroll
        for (int v = 0; v < NC; ++v) xp[s][v] = XP[(v * S + s) * B + tid];
#pragma unroll
        for (int r = 0; r < NR; ++r) yp[s][r] = YP[(r * S + s) * B + tid];
      }
    }
  };
  // (DVH_BAND_PROBE) stamps label the segment they end; a segment is added at the NEXT stamp, so that no stamp waits
  // for its own s_memtime (a stamp's value is first used after the barrier that follows it)
  unsigned pacc[5] = {0u, 0u, 0u, 0u, 0u};
  unsigned long long pt1 = 0ull, pt2 = 0ull;
  auto pstamp = [&](int seg) __attribute__((always_inline)) {
    if constexpr (DVH_BAND_PROBE) {
      const unsigned long long t = probe_clock();
      if (seg < 0) {
        pt1 = pt2 = t;
      } else {
        pacc[(seg + 4) % 5] += (unsigned)(pt1 - pt2);
        pt2 = pt1;
        pt1 = t;
      }
    }
  };
  auto iterate = [&](auto chk_tag, auto w0_tag) __attribute__((always_inline)) {
    constexpr bool CHECK = decltype(chk_tag)::value;
    constexpr bool W0 = decltype(w0_tag)::value;
    if constexpr (W0 && DVH_BAND_PRIO) __builtin_amdgcn_s_setprio(DVH_BAND_PRIO);
    pstamp(4);  // (the check code since the last iteration, or the loop entry)
    if (kin - kbase >= kWave) {
      kbase = kin;
      hw = hload(kin);
    }
    const double cb = readlane_f64(hw, kin - kbase), ca = 1.0 - cb;
    mv0 = mv1 = mv2 = mv3 = 0.0;
    mvb0 = mvb1 = 0.0;
    // ---------------- primal half-step (reflected Halpern, rho = 1)
    double kx[S][NR];  // own-lane part of K x-bar for the dual half-step
    // the dual update of step s's r-th row from kx (row 0, SOE, is an equality; DCM / ICE rows are >=: duals >= 0)
    auto row_step = [&](int s, int r) __attribute__((always_inline)) {
      if (!CHECK && r == 0) {  // equality row, no image needed: 2 (y - sigma Kx) - y = y - 2 sigma Kx
        y[s][0] = fma(ca, fma(sigma2n, kx[s][0], y[s][0]), cb * ayv(s, 0));
        return;
      }
      double p1 = fma(-sigma, kx[s][r], y[s][r]);
      if (r > 0) p1 = vmax(p1, 0.0);
      if (CHECK) {
        const double d = y[s][r] - p1, da = p1 - ayv(s, r);
        mv2 += d * d;
        mv3 += da * da;
        if constexpr (LI) {
          const int i = row_of(s, r);
          if (i >= 0) yim[opaque(i)] = p1;
        } else {
          YP[(r * S + s) * B + tid] = p1;
        }
      }
      y[s][r] = fma(ca, fma(2.0, p1, -y[s][r]), cb * ayv(s, r));
    };
    {
      double ta0 = 0.0, ta1 = 0.0;
      if constexpr (W0 && kTauWaveSums) {
        ta0 = tau_waves();
      } else if constexpr (W0) {  // (0 + a == a: the first partials start the two chains)
        ta0 = TP[lane];
        if (NW > 1) ta1 = TP[kWave + lane];
#pragma unroll
        for (int r = 2; r < NW; r += 2) {
          ta0 += TP[r * kWave + lane];
          if (r + 1 < NW) ta1 += TP[(r + 1) * kWave + lane];
        }
      }
      double kty[S][NC], xb[S][NC];
      const double ysp = YS[tid];
#pragma unroll
      for (int s = 0; s < S; ++s) ktr_c(s, y[s], s == 0 ? ysp : y[s > 0 ? s - 1 : 0][0], kty[s]);
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int v = 0; v < NC; ++v) {  // branch-free: padding steps have c = lo = hi = 0 and stay at 0
          double p1;
          if constexpr (BOX) {
            p1 = fma_clamp01(v < 3 ? tj[s][v < 3 ? v : 0] : ro(v - 1, s), kty[s][v], x[s][v]);
          } else {
            const double lo = v == 2 ? loe[s] : 0.0;
            p1 = vmin(vmax(fma(tau, kty[s][v], x[s][v]), lo), hib(s, v));
          }
          xb[s][v] = fma(2.0, p1, -x[s][v]);
          if (CHECK) {
            double d = x[s][v] - p1, da = p1 - axv(s, v);
            if constexpr (BOX && kBoxRescale) {  // movements in x units: w^2 = tau_bs / step (0 for a fixed column)
              const double st = v < 3 ? tj[s][v < 3 ? v : 0] : ro(v - 1, s);
              const double iw = st > 0.0 ? (double)__builtin_amdgcn_rcp(st) : 0.0;
              mvb0 = fma(d * d, iw, mvb0);
              mvb1 = fma(da * da, iw, mvb1);
            } else {
              if constexpr (BOX) {  // movements in x units
                const double wv = wcol(s, v);
                d *= wv;
                da *= wv;
              }
              mv0 += d * d;
              mv1 += da * da;
            }
            if constexpr (LI) {
              if (val[s]) xim[opaque(col(s, v))] = p1;
            } else {
              XP[(v * S + s) * B + tid] = p1;
            }
          }
          x[s][v] = fma(ca, xb[s][v], cb * axv(s, v));
        }
      }
      XE[tid] = xb[0][2];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        kown_q(s, xb[s], kx[s]);
        if (s < S - 1) kfin_next(s, kx[s], xb[s < S - 1 ? s + 1 : s][2]);  // the next step is the lane's own
      }
      if constexpr (W0 && kTauWaveSums) {
        tau_update(ta0, ca, cb, chk_tag);
      } else if constexpr (W0) {
        tau_update(uniform(wave_sum_dpp(ta0 + ta1)), ca, cb, chk_tag);
      } else {
        if (wid == 0 && J > 1) tau_update(tau_kt(), ca, cb, chk_tag);
      }
    }
    pstamp(0);
    if constexpr (!W0 && (DVH_BAND_PIN_KX > 1 || (DVH_BAND_PIN_KX == 1 && ICE))) {  // (DVH_BAND_PIN_KX) K x-bar first
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int r = 0; r < NR; ++r) asm volatile("" ::"v"(kx[s][r]));
    }
    lds_barrier();
    if constexpr (W0 && DVH_BAND_PRIO) __builtin_amdgcn_s_setprio(0);
    pstamp(1);
    // ---------------- dual half-step
    {
      if constexpr (DVH_BAND_PRIO_DUAL) __builtin_amdgcn_s_setprio(DVH_BAND_PRIO_DUAL);
      // every LDS read of the half-step first (the next lane's ene, the tau columns' x-bar), before any LDS store:
      // issued together, one wait instead of one per read
      const double xen = XE[tid + 1];
      double xtv[S];
#pragma unroll
      for (int s = 0; s < S; ++s) xtv[s] = lds_ld(xta[s]);
      kfin_next(S - 1, kx[S - 1], xen);
      // the >= rows first: their duals feed the tau partials, whose wave reduction then has the SOE rows' work
      // beside it
#pragma unroll
      for (int s = 0; s < S; ++s) {
        kx[s][1] = fma(kd[s][2], xtv[s], kx[s][1]);  // kfin_tau
#pragma unroll
        for (int r = 1; r < ((DVH_BAND_LATE_ICE && ICE && !W0) ? 2 : NR); ++r) row_step(s, r);
      }
      if (J > 0) tau_parts_of(y);
      if constexpr (DVH_BAND_PRIO_DUAL) __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int s = (DVH_BAND_LATE_SOE && !W0) ? S - 1 : 0; s < S; ++s) row_step(s, 0);
      YS[tid + 1] = y[S - 1][0];
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
    pstamp(2);
    if constexpr (W0 && DVH_BAND_PIN_BLEND) {  // (see DVH_BAND_PIN_BLEND) this iteration's blends before the barrier
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int v = 0; v < NC; ++v) asm volatile("" ::"v"(x[s][v]));
#pragma unroll
        for (int r = 0; r < NR; ++r) asm volatile("" ::"v"(y[s][r]));
      }
    }
    lds_barrier();
    if constexpr (DVH_BAND_LATE_SOE && !W0) {  // (DVH_BAND_LATE_SOE) the lane-local SOE rows, after the barrier
#pragma unroll
      for (int s = 0; s < S - 1; ++s) row_step(s, 0);
    }
    if constexpr (DVH_BAND_LATE_ICE && ICE && !W0) {  // (DVH_BAND_LATE_ICE) the ICE rows, after the barrier
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int r = 2; r < NR; ++r) row_step(s, r);
    }
    pstamp(3);
  };

  using F = std::integral_constant<bool, false>;
  using Tt = std::integral_constant<bool, true>;
  pstamp(-1);
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
    const bool last = it + chk > o.max_iters;
    bool kkt = (--kk_ == 0) || last;
    if (kkt) kk_ = kkt_every;
    // the ICE form reduces the round-3 set (no dual-residual term in its objective gate): the extra value cost it 6 %
    // on config 5 at unchanged iterations (register pressure of its check path; profiles/r04ab_ab_kkt_rdx.log)
    constexpr int NRED = (ICE && DVH_KKT_RDX) ? kNRed - 1 : kNRed;
    double acc[NRED];
    acc[0] = fma(tau_bs, mvb0, mv0);  // (mvb0 = mvb1 = 0 without kBoxRescale)
    acc[1] = fma(tau_bs, mvb1, mv1);
    acc[2] = mv2;
    acc[3] = mv3;
#pragma unroll
    for (int u = 4; u < NRED; ++u) acc[u] = 0.0;
    double r = 0.0;
    if constexpr (GATE) {
      // predicted KKT gate: the restart sums first; a due check runs only if the last check's worst ratio to eps,
      // scaled by the fixed-point residual's decrease since then, is within kkt_predict (or 4 were skipped)
      double acc4[4] = {acc[0], acc[1], acc[2], acc[3]};
      block_sum1<B, 4, true>(acc4, red);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = acc4[u];
      r = usc<ICE>(sqrt(pw * acc[0] + acc[2] / pw));
      if (kkt && !last && kkt_gate_skip(o, gate, r)) {
        kkt = false;
        ++gate.skip;
      }
    }
    if (kkt) {
      // (kkt_prefetch) the single-precision factors of the lane's columns and rows, loaded together first: one wait
      // for all of them, behind the image reads and the barrier below
      // (branch-free: a padding step / absent row loads the window's first entry and discards it; the indices are
      // formed here from an opaque thread index, so that they are not hoisted out of the loop and held)
      float fcl[S][NC], frl[S][NR], fspl = 1.0f;
      if constexpr (kkt_prefetch<ICE>()) {
        const int to = S * opaque(tid);
        const float* fcw = w.fc + W.wn;
        const float* frw = w.fr + W.wm;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const bool vs = to + s < T;
#pragma unroll
          for (int v = 0; v < NC; ++v) {
            const int j = v < 3 ? v * T + to + s : (v == 3 ? CE : CO) + to + s;
            const float f = fcw[vs ? j : 0];
            fcl[s][v] = vs ? f : 1.0f;
          }
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = r == 0 ? (vs ? to + s + 1 : -1) : r == 1 ? DRL[s * B + tid] : (vs ? (r == 2 ? ra[s] : rb[s]) : -1);
            const float f = frw[i >= 0 ? i : 0];
            frl[s][r] = i >= 0 ? f : 1.0f;
          }
        }
        const int lo_ = (to / S) & (kWave - 1);  // (the lane, from the opaque thread index)
        const float ft = fcw[tlane ? 3 * T + lo_ : 0], fi = frw[0];
        fspl = tlane ? ft : ilane ? fi : 1.0f;
      }
      // images of T(z_k) in XE / XT / YS / TP (rewritten from z after the check)
      double xp[S][NC], yp[S][NR];
      load_images(xp, yp);
      XE[tid] = xp[0][2];
      YS[tid + 1] = yp[S - 1][0];
      if (ilane) YS[0] = sp[2];
      if (tlane) XT[lane] = sp[5];
      if (J > 0) tau_parts_of(yp);
      lds_barrier();
      auto col_kkt = [&](int j, double kt, double cj, double loj, double hij, double xj, float fpre) {
        const float fd = kkt_prefetch<ICE>() ? fpre : w.fc[W.wn + opaque(j)];
        if constexpr (NRED > kRdx && DVH_KKT_RDX) {
          const ColKktX r = col_kkt_fn_x<kkt_inline<ICE>()>(kt, cj, loj, hij, xj, fd);
          acc[5] += r.rd2;
          acc[6] += r.cx;
          acc[8] += r.bt;
          acc[kRdx] += r.rdx;
        } else {
          const ColKkt r = col_kkt_fn<kkt_inline<ICE>()>(kt, cj, loj, hij, xj, fd);
          acc[5] += r.rd2;
          acc[6] += r.cx;
          acc[8] += r.bt;
        }
      };
      auto row_kkt = [&](int i, double kv, double qi, double yi, bool ge, float fpre) {
        const float fd = kkt_prefetch<ICE>() ? fpre : w.fr[W.wm + opaque(i)];
        const RowKkt r = row_kkt_fn<kkt_inline<ICE>()>(kv, qi, yi, fd, ge);
        acc[4] += r.rp2;
        acc[7] += qi * yi;
        acc[9] += r.y2;
      };
      const double ysp = YS[tid];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        double kt[NC];
        ktr(s, yp[s], s == 0 ? ysp : yp[s > 0 ? s - 1 : 0][0], kt);
        if (val[s]) {
#pragma unroll
          for (int v = 0; v < NC; ++v) {
            if constexpr (BOX)  // the primed LP: box [0, 1]
              col_kkt(col(s, v), kt[v], cof(s, v), 0.0, 1.0, xp[s][v], fcl[s][v]);
            else
              col_kkt(col(s, v), kt[v], cof(s, v), v == 2 ? loe[s] : 0.0, hib(s, v), xp[s][v], fcl[s][v]);
          }
        }
      }
      if (wid == 0 && J > 0) {
        const double ktt = tau_kt();
        if (tlane) col_kkt(3 * T + lane, ktt, sp[2], sp[3], sp[4], sp[5], fspl);
      }
      const double xen = XE[tid + 1];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        double kv[NR];
        kown(s, xp[s], kv);
        kfin_next(s, kv, s == S - 1 ? xen : xp[s < S - 1 ? s + 1 : s][2]);
        kfin_tau(s, kv);
        const int t = t0 + s;
        if (val[s]) row_kkt(t + 1, kv[0], qv(s, 0), yp[s][0], false, frl[s][0]);
        const int dr_ = DRL[s * B + tid];
        if (dr_ >= 0) row_kkt(dr_, kv[1], qv(s, 1), yp[s][1], true, frl[s][1]);
        if constexpr (LI) {  // this check's T(z_k), unscaled, as the outputs
          if (val[s]) {
#pragma unroll
            for (int v = 0; v < NC; ++v) {
              const int j = opaque(col(s, v));
              xo_g[j] = xp[s][v] * dcf(j);
            }
          }
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int i = row_of(s, r);
            if (i >= 0) yo_g[opaque(i)] = yp[s][r] * drf(opaque(i));
          }
        }
        if (ICE && val[s]) {
          row_kkt(ra[s], kv[2], rhs(s, 2), yp[s][2], true, frl[s][NR > 2 ? 2 : 0]);
          row_kkt(rb[s], kv[3], rhs(s, 3), yp[s][3], true, frl[s][NR > 3 ? 3 : 0]);
        }
      }
      if (ilane) row_kkt(0, sp[4] * XE[0], sp[3], sp[2], false, fspl);
    }
    if constexpr (GATE) {
      if (kkt) {  // the KKT sums in the slots after the restart sums' (red is not reused before a barrier)
        double acc6[NRED - 4];
#pragma unroll
        for (int u = 4; u < NRED; ++u) acc6[u - 4] = acc[u];
        block_sum1<B, NRED - 4, true>(acc6, red + 4 * NW);
#pragma unroll
        for (int u = 4; u < NRED; ++u) acc[u] = acc6[u - 4];
      }
    } else if (kkt) {
      block_sum1<B, NRED, true>(acc, red);
    } else {
      double acc4[4] = {acc[0], acc[1], acc[2], acc[3]};
      block_sum1<B, 4, true>(acc4, red);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = acc4[u];
    }
    if constexpr (!GATE) r = usc<ICE>(sqrt(pw * acc[0] + acc[2] / pw));
    if (kkt) {
      const double pobj = usc<ICE>(acc[6] + c0), dobj = usc<ICE>(acc[7] + acc[8] + c0);
      const double pres = usc<ICE>(sqrt(acc[4]) / (1.0 + sgpr_fresh<ICE>(qnorm)));
      const double dres = usc<ICE>(sqrt(acc[5]) / (1.0 + sgpr_fresh<ICE>(cnorm)));
      const double gap = usc<ICE>(fabs(pobj - dobj) / (1.0 + fabs(pobj) + fabs(dobj)));
      if (tid == 0) {
        fin[0] = pobj;
        fin[1] = pres;
        fin[2] = dres;
        fin[3] = gap;
      }
      if (kkt_done(o, pres, dres, gap, pobj, dobj, acc[4], acc[9], (NRED > kRdx && DVH_KKT_RDX) ? acc[kRdx] : 0.0)) {
        status = kOptimal;
        break;
      }
      if constexpr (GATE) {
        gate.note(pres, dres, gap, o.eps, r);
        gate.q = usc<ICE>(gate.q);
      }
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
      if (ddx > 1e-10 && ddy > 1e-10) pw = uniform(pw_update<!ICE>(ddy / ddx, pw, o.theta));
      tau = uniform(eta / pw);
      sigma = uniform(eta * pw);
      sigma2n = uniform(-2.0 * sigma);
      box_steps_rescale();
      double xp[S][NC], yp[S][NR];
      load_images(xp, yp);
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int v = 0; v < NC; ++v) {
          x[s][v] = xp[s][v];
          if constexpr (LA)
            XA[(v * S + s) * B + tid] = x[s][v];
          else
            xa[s][v] = x[s][v];
        }
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
          y[s][rr] = yp[s][rr];
          if constexpr (LA)
            YA[(rr * S + s) * B + tid] = y[s][rr];
          else
            ya[s][rr] = y[s][rr];
        }
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
      YS[tid + 1] = y[S - 1][0];
      if (ilane) YS[0] = sp[0];
      if (J > 0) tau_parts_of(y);
      lds_barrier();
    }
    // (a restart check that neither restarts nor checks KKT rewrote no shared value: the next iteration reads what the
    // check iteration wrote before its barriers, and `red` is next written two barriers later -- no barrier here)
  }
  // outputs: the last check's T(z_k), unscaled (the lean form wrote them at that check)
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (LI || !val[s]) continue;
    const int t = t0 + s;
#pragma unroll
    for (int v = 0; v < NC; ++v) {
      const int j = col(s, v);
      if constexpr (BOX) {  // x = lo + w x' (clipped to the box against the rounding), then unscaled
        const double d = dcf(j), lo = lraw[j] / d, hv = uraw[j] / d;
        double wv;
        if constexpr (kNoWidths) {  // the set-up's width, by the set-up's operations
          wv = hv - (v == 2 ? lo : 0.0);
          if (!(wv >= 0x1p-500)) wv = 0.0;
        } else {
          wv = wbox[j];
        }
        xo_g[j] = fmin(fmax(fma(wv, XP[(v * S + s) * B + tid], lo), lo), hv) * d;
      } else {
        xo_g[j] = XP[(v * S + s) * B + tid] * dcf(j);
      }
    }
    yo_g[t + 1] = YP[s * B + tid] * drf(t + 1);
    const int dr_ = DRL[s * B + tid];
    if (dr_ >= 0) yo_g[dr_] = YP[(S + s) * B + tid] * drf(dr_);
    if (ICE) {
      yo_g[ra[s]] = YP[(2 * S + s) * B + tid] * drf(ra[s]);
      yo_g[rb[s]] = YP[(3 * S + s) * B + tid] * drf(rb[s]);
    }
  }
  if (tlane) xo_g[3 * T + lane] = sp[5] * dcf(3 * T + lane);
  if (ilane) yo_g[0] = sp[2] * drf(0);
  if constexpr (DVH_BAND_PROBE) {
    pstamp(4);
    pacc[4] += (unsigned)(pt1 - pt2);
    unsigned hw = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    __syncthreads();
    if (lane == 0) {
      for (int u = 0; u < 5; ++u) xo_g[6 * wid + u] = (double)pacc[u];
      xo_g[6 * wid + 5] = (double)hw;
    }
  }
  if (tid == 0) {
    b.istats[2 * k] = status;
    b.istats[2 * k + 1] = it;
    for (int u = 0; u < 4; ++u) b.stats[4 * k + u] = fin[u];
  }
}

// Persistent form (PERSIST; the three-step battery form): the grid is the device's resident workgroup slots (two per CU),
// and each workgroup takes the next window from an atomic counter until the list is exhausted, so a slot freed by a
// short window takes the next one at once.  One workgroup per window left the slots to the hardware dispatcher,
// which deals workgroups in order round-robin over the XCDs: with durations that vary window to window (warm
// iterations 200 .. 10,000) the in-order dispatch leaves slots idle.  Measured: the bench's windows ran 7-8 % faster
// when launched sorted by their own iteration counts (either direction, profiles/r04r_ab_launch_order.log), a
// synthetic kernel of random durations lost 20 % to the sorted order (scripts/probe_dispatch.hip,
// profiles/r04t_probe_dispatch.log: 33.5 vs 28.2 ms, persistent 29.9), and the persistent band kernel runs the
// bench's PDHG in 467 vs 478 ms (profiles/r04u_ab_band_queue.log).  The persistent instantiations (the three-step
// battery form and the ICE form) are compiled in dvh_band_persist.hip without machine-level loop-invariant code motion:
// built with it, the window setup's invariants were hoisted out of the loop over windows and spilled (12.6 % slower per
// iteration, and the ICE form 61k vs 91k windows/s on config 5).  Now the battery form's PDHG runs 441 vs 459 ms and
// config 5 112.7k vs 95.6k windows/s (profiles/r04al_band_persist_nolicm.log, r04an_ab_ice_queue.log); the one-step
// battery form stays one workgroup per window.  Every workgroup leaves once the counter passes the list (the counter
// zeroed on the stream before the launch).
struct BandArgs {
  Batch b;
  Work w;
  Chunk ch;
  Opts o;
  const int32_t* list;  // global window indices, or null: the chunk
  int count;            // windows to solve (list entries, or the chunk's)
  int32_t* queue;       // work-queue counter (PERSIST), zeroed before the launch
};
template <int B, int S, bool ICE, int LF, int WPS, bool GATE, bool BOX, bool PERSIST>
__global__ __launch_bounds__(B, WPS) void pdhg_band_kernel(const BandArgs args) {
  if constexpr (!PERSIST) {
    const int i = blockIdx.x;
    band_window<B, S, ICE, LF, WPS, GATE, BOX>(args.b, args.w, args.ch, args.o,
                                               args.list ? args.list[i] : args.ch.first + i, threadIdx.x);
  } else {
    __shared__ int32_t next;
    for (;;) {
#if defined(__HIP_DEVICE_COMPILE__)
      // The arguments are read through a kernarg pointer the compiler cannot see through, once per window: read as
      // `args`, their ~70 scalar loads were hoisted out of this loop and kept live across the window (SGPRs spilled
      // to VGPR lanes, 56 dwords of VGPRs to scratch; 12.6 % slower per iteration than one workgroup per window at
      // equal durations, profiles/r04ak_band_queue_iter.log).  Laundered, each window reloads what it uses.
      using KArgs = const __attribute__((address_space(4))) BandArgs*;
      KArgs kp = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
      asm volatile("" : "+s"(kp));
      const BandArgs& args = *(const BandArgs*)kp;
#endif
      // wave 0 takes the next window in a wave-uniform branch, the whole wave in the atomic (lane 0 adds 1, the others
      // 0): a lane-0-only atomic inside the loop is structurized into an inner loop whose barriers the waves do not
      // reach in step (the workgroups hang: scripts/probe_dispatch.hip)
      if (__builtin_amdgcn_readfirstlane(threadIdx.x) < kWave)
        next = __builtin_amdgcn_readfirstlane(atomicAdd(args.queue, (threadIdx.x & (kWave - 1)) == 0 ? 1 : 0));
      __syncthreads();
      const int i = __builtin_amdgcn_readfirstlane(next);  // uniform: the loop's exit is a scalar branch
      __syncthreads();  // (every wave has read it before wave 0 takes the next one)
      if (i >= args.count) return;
      int tid = threadIdx.x;
#if defined(__HIP_DEVICE_COMPILE__)
      asm volatile("" : "+v"(tid));  // (likewise what the window derives from its thread index)
#endif
      band_window<B, S, ICE, LF, WPS, GATE, BOX>(args.b, args.w, args.ch, args.o,
                                                 args.list ? args.list[i] : args.ch.first + i, tid);
    }
  }
}

#ifndef DVH_BANDI_LF
#define DVH_BANDI_LF 0
#endif
#ifndef DVH_BAND3_LF
#define DVH_BAND3_LF kLfCosts
#endif
template <int B, int S, bool ICE, int LF, int WPS, bool GATE, bool BOX, bool PERSIST>
hipError_t launch_band_one_q(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s,
                             const int32_t* list, int nlist, int* variant_out) {
  static_assert(B * S == kBandSteps, "every form covers T <= kBandSteps");
  const size_t lds = band_lds_bytes(B, S, ICE, LF);
  auto kern = pdhg_band_kernel<B, S, ICE, LF, WPS, GATE, BOX, PERSIST>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (getenv("DVH_BAND_OCC")) {  // residency diagnostics (A/B helper)
    int nb = -1, dev = 0;
    hipGetDevice(&dev);
    hipDeviceProp_t pr;
    hipGetDeviceProperties(&pr, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, B, lds);
    hipFuncAttributes fa;
    hipFuncGetAttributes(&fa, (const void*)kern);
    fprintf(stderr, "band<%d,%d,%d,%d,gate %d,box %d,persist %d>: lds %zu B, blocks/CU %d, lds/CU %zu, regs %d, local %zu\n",
            B, S, (int)ICE, LF, (int)GATE, (int)BOX, (int)PERSIST, lds, nb, (size_t)pr.maxSharedMemoryPerMultiProcessor,
            fa.numRegs, (size_t)fa.localSizeBytes);
  }
  const int count = list ? nlist : ch.count;
  if (count <= 0) return hipSuccess;
  int grid = count;
  if (PERSIST) {  // every resident slot (workgroups per CU at this form x CUs), or fewer
    // measured once per handle (each handle belongs to one device and one host thread at a time; Work::slots)
    int& slots = w.slots[(ICE ? 4 : 0) + (GATE ? 2 : 0) + (BOX ? 1 : 0)];
    if (slots <= 0) {
      int nb = 0, cus = 0, dev = 0;
      if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
      if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, B, lds)) != hipSuccess) return e;
      if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
      slots = std::max(1, nb) * std::max(1, cus);
    }
    // DVH_BAND_RESERVE = k: leave 2k workgroup slots to other kernels, e.g. an all-gather issued on another stream
    // after this grid launched, which otherwise waits for the grid's tail (scripts/probe_overlap.py,
    // profiles/r05i_overlap_reserve*.log: k = 32 lets a 2 GiB copy run beside the grid at +12.6 % band time)
    static const int reserve = [] { const char* e = getenv("DVH_BAND_RESERVE"); return e ? std::max(0, atoi(e)) : 0; }();
    grid = std::min(count, std::max(1, slots - 2 * reserve));
    if ((e = hipMemsetAsync(w.queue, 0, sizeof(int32_t), s)) != hipSuccess) return e;
  }
  const BandArgs args{b, w, ch, o, list, count, w.queue};
  hipLaunchKernelGGL(kern, dim3(grid), dim3(B), lds, s, args);
  if (variant_out) *variant_out = 9000000 + 1000 * (S - 1) + (ICE ? 100 : 0) + B / kWave;
  return hipGetLastError();
}
template <int B, int S, bool ICE, int LF, int WPS, bool GATE, bool BOX>
hipError_t launch_band_one_g(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s,
                             const int32_t* list, int nlist, int* variant_out) {
  if constexpr (S == 3 && !ICE) {  // the persistent form (DVH_BAND_QUEUE=0: one workgroup per window, A/B)
    static_assert(B == kBandSteps / 3 && LF == DVH_BAND3_LF && WPS == 2, "dvh_band_persist.hip instantiates this form");
    const char* q = getenv("DVH_BAND_QUEUE");
    if (!(q && atoi(q) == 0)) return launch_band_persist(GATE, BOX, b, w, ch, o, s, list, nlist, variant_out);
  }
  if constexpr (ICE) {  // the ICE form's persistent grid (DVH_BAND_QUEUE=0 or DVH_BAND_QUEUE_ICE=0: off, A/B)
    static_assert(B == kBandSteps && S == 1 && LF == DVH_BANDI_LF && WPS == 3, "dvh_band_persist_ice.hip instantiates this form");
    const char* q = getenv("DVH_BAND_QUEUE");
    const char* qi = getenv("DVH_BAND_QUEUE_ICE");
    if (!(q && atoi(q) == 0) && !(qi && atoi(qi) == 0))
      return launch_band_persist_ice(GATE, BOX, b, w, ch, o, s, list, nlist, variant_out);
  }
  return launch_band_one_q<B, S, ICE, LF, WPS, GATE, BOX, false>(b, w, ch, o, s, list, nlist, variant_out);
}
template <int B, int S, bool ICE, int LF, int WPS, bool BOX = false>
hipError_t launch_band_one(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s,
                           const int32_t* list, int nlist, int* variant_out) {
  if (o.kkt_predict > 0)
    return launch_band_one_g<B, S, ICE, LF, WPS, true, BOX>(b, w, ch, o, s, list, nlist, variant_out);
  return launch_band_one_g<B, S, ICE, LF, WPS, false, BOX>(b, w, ch, o, s, list, nlist, variant_out);
}

}  // namespace

// Forms of the battery (non-ICE) band kernel.  form 3 (default): 256 threads = one wave per SIMD, three steps per
// lane, <= 256 VGPRs = 2 waves per SIMD, so two windows share every CU (a 384-thread, two-step form with 3 waves
// per SIMD was measured to run one window per CU in practice: its 6 waves cannot be placed 3 / 3 / 3 / 3); the
// costs / right-hand sides in LDS keep its three steps' state in 256 VGPRs without spills in the iteration, and the
// setup-only ints share the check images' LDS so that two windows fit one CU's LDS (74 KB each).  Measured
// (profiles/r02x_band_forms.log): 0.51 vs 0.69 us per window-iteration per CU; with the images in the global
// workspace (kLfImages) 5 % slower and 10x the HBM writes, with the anchors in LDS too (kLfAnchors) 8 % slower.
// form 1: 768 threads, one step per lane, 12 waves, one window per CU (A/B, dvh_set_kernel_path 3).  The LP-relaxed
// ICE windows keep the one-step form (twice the per-step state).
#if DVH_BAND_PERSIST_TU == 1
// The persistent forms (three-step battery: dvh_band_persist.hip, DVH_BAND_PERSIST_TU 1; ICE: dvh_band_persist_ice.hip, 2),
// each this file in a translation unit of its own, compiled without
// machine-level loop-invariant code motion: hoisted out of the persistent loop, the window setup's invariants stayed live
// across every window's iterations (56 spilled dwords, 12.6 % slower per iteration than one workgroup per window at
// equal durations; 1.6 % without the hoisting, profiles/r04al_band_persist_nolicm.log).  The one-workgroup forms keep
// the hoisting (this build of them is 1.4 % slower per iteration).
hipError_t launch_band_persist(bool gate, bool box, const Batch& b, const Work& w, const Chunk& ch, const Opts& o,
                               hipStream_t s, const int32_t* list, int nlist, int* variant_out) {
  constexpr int B = kBandSteps / 3;
  if (gate) {
    if (box) return launch_band_one_q<B, 3, false, DVH_BAND3_LF, 2, true, true, true>(b, w, ch, o, s, list, nlist, variant_out);
    return launch_band_one_q<B, 3, false, DVH_BAND3_LF, 2, true, false, true>(b, w, ch, o, s, list, nlist, variant_out);
  }
  if (box) return launch_band_one_q<B, 3, false, DVH_BAND3_LF, 2, false, true, true>(b, w, ch, o, s, list, nlist, variant_out);
  return launch_band_one_q<B, 3, false, DVH_BAND3_LF, 2, false, false, true>(b, w, ch, o, s, list, nlist, variant_out);
}
#elif DVH_BAND_PERSIST_TU == 2
hipError_t launch_band_persist_ice(bool gate, bool box, const Batch& b, const Work& w, const Chunk& ch, const Opts& o,
                                   hipStream_t s, const int32_t* list, int nlist, int* variant_out) {
  constexpr int B = kBandSteps;
  if (gate) {
    if (box) return launch_band_one_q<B, 1, true, DVH_BANDI_LF, 3, true, true, true>(b, w, ch, o, s, list, nlist, variant_out);
    return launch_band_one_q<B, 1, true, DVH_BANDI_LF, 3, true, false, true>(b, w, ch, o, s, list, nlist, variant_out);
  }
  if (box) return launch_band_one_q<B, 1, true, DVH_BANDI_LF, 3, false, true, true>(b, w, ch, o, s, list, nlist, variant_out);
  return launch_band_one_q<B, 1, true, DVH_BANDI_LF, 3, false, false, true>(b, w, ch, o, s, list, nlist, variant_out);
}
#else
hipError_t launch_pdhg_band(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s, bool ice,
                            int form, bool box, const int32_t* list, int nlist, int* variant_out) {
  if (ice) {
    if (box) return launch_band_one<kBandSteps, 1, true, DVH_BANDI_LF, 3, true>(b, w, ch, o, s, list, nlist, variant_out);
    return launch_band_one<kBandSteps, 1, true, DVH_BANDI_LF, 3>(b, w, ch, o, s, list, nlist, variant_out);
  }
  if (form == 1) {
    if (box) return launch_band_one<kBandSteps, 1, false, 0, 3, true>(b, w, ch, o, s, list, nlist, variant_out);
    return launch_band_one<kBandSteps, 1, false, 0, 3>(b, w, ch, o, s, list, nlist, variant_out);
  }
  if (box) return launch_band_one<kBandSteps / 3, 3, false, DVH_BAND3_LF, 2, true>(b, w, ch, o, s, list, nlist, variant_out);
  return launch_band_one<kBandSteps / 3, 3, false, DVH_BAND3_LF, 2>(b, w, ch, o, s, list, nlist, variant_out);
}
#endif

}  // namespace dvh

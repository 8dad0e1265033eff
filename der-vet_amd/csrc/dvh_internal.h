// Internal declarations shared by the C-ABI layer (dvh_api.cpp) and the HIP kernels (dvh_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

struct dvh_window_series;  // include/dervet_hip.h

namespace dvh {

constexpr int kWave = 64;
constexpr int kLongRow = 32;   // CSR rows longer than this are reduced by a whole wave
constexpr int kLMax = 64;      // long rows per matrix per window handled on chip
constexpr int kScal = 16;      // per-window scalars written by the setup kernel
constexpr int kHalpernTab = 65536;  // table of Halpern weights 1/(k+2)
constexpr int kSmallMax = 4096;     // windows with n or m above this go to the medium tier or the large-LP path
// Medium tier (dvh_chain.hip): battery windows of up to kPMax segments of kChainB steps, one workgroup per segment.
// Windows of up to kChainMedMax segments run as a batch (teams inside one XCD where they fit); longer ones (the
// 5-minute annual window of BASELINE config 3: T = 105,120, 137 segments) run in a launch of their own, one team
// spanning the chip.
constexpr int kChainB = 768;
constexpr int kPMax = 192;
constexpr int kChainMedMax = 16;
constexpr int kChainJMax = 256;     // tau (demand) columns per medium window
constexpr int kChainJSeg = 4;       // tau columns per segment
// plan words per window: [0] P, [1] T, [2] J, [3] k, [kPlanStart + s] first step of segment s (P + 1 entries),
// per (segment s, slot u): the tau column [kPlanSlot + 4 s + u] (-1: none) and the contiguous range of segments that
// share it [kPlanLo / kPlanHi + 4 s + u] (every segment of the range holds the column in a slot)
constexpr int kPlanStart = 4;
constexpr int kPlanSlot = kPlanStart + kPMax + 4;
constexpr int kPlanLo = kPlanSlot + kChainJSeg * kPMax;
constexpr int kPlanHi = kPlanLo + kChainJSeg * kPMax;
constexpr int kPlanInts = kPlanHi + kChainJSeg * kPMax;
// windows whose n reaches this are set up grid-wide (setup_long, dvh_chain.hip): the one-workgroup setup kernel keeps
// n + 1 transpose cursors in LDS
constexpr int kMedSetupNMax = 40000;

// Kernel-side copy of dvh_options (POD, passed by value).
struct Opts {
  double eps, step_safety, rho, b_suff, b_nec, b_art, theta;
  double eps_obj;      // objective-error termination (dvh_options.eps_obj; 0 = off)
  int max_iters, check_every, kkt_every, ruiz_iters, power_iters;
  int setup_segments;  // set by launch_setup
  int small_max;       // setup skips (scal[6] = 2) windows with n or m above this
  int warm;            // start from the (unscaled) x / y in the output buffers (band kernel; others cold)
  int kkt_predict;     // dvh_options.kkt_predict (band kernel; 0 = off)
};

// Inputs of one chunk of the packed batch (device pointers, global offsets from desc).
struct Batch {
  const int64_t* desc;
  const int32_t* indptr;
  const int32_t* indices;
  const double* data;
  const double* c;
  const double* c0;
  const double* q;
  const double* l;
  const double* u;
  double* x;
  double* y;
  double* stats;
  int32_t* istats;
};

// Per-chunk device workspace.  Window k of the chunk uses offsets (desc offsets - chunk base).
struct Work {
  int32_t* tptr;    // [sum(n+1)]   K^T row pointers        at (off_n - base_n) + (k - first)
  int32_t* tind;    // [sum nnz]    K^T column (= K row) ids
  double* tval;     // [sum nnz]    scaled K^T values
  double* kval;     // [sum nnz]    scaled K values
  int32_t* rowof;   // [sum nnz]    K entry -> row
  int32_t* perm;    // [sum nnz]    K entry -> K^T slot
  double* dr;       // [sum m]
  double* dc;       // [sum n]
  double* cs;       // [sum n]  Dc c
  double* ls;       // [sum n]  l / Dc
  double* us;       // [sum n]  u / Dc
  double* qs;       // [sum m]  Dr q
  double* vbuf;     // [sum n]
  double* wbuf;     // [sum m]
  double* tmpc;     // [sum n]
  double* tmpr;     // [sum m]
  int32_t* longk;   // [count * kLMax]  long rows of K
  int32_t* longt;   // [count * kLMax]  long rows of K^T (dense columns, e.g. the DCM tau)
  const double* hinv;  // [kHalpernTab] 1 / (k + 2), k = 0.. (Halpern anchor weights, exact IEEE quotients)
  double* scal;     // [count * kScal]  eta, w0, ||c||, ||q||, nlong(K), nlong(K^T), flag, ||K||,
                    //   max short row len K, K^T (<= 8), #rows > 8 in K, K^T
  float* fc;        // [sum n]  Dc rounded to single precision (the band kernel's KKT checks; written by the band
                    //          kernels, whose factors stay within [2^-100, 2^100])
  float* fr;        // [sum m]  Dr rounded to single precision
  int32_t* queue;   // [1] the band kernels' work-queue counter (zeroed before each launch)
  int* slots;       // HOST [kPersistForms]: resident workgroup slots of each persistent band form on this handle's
                    //   device (0: not measured yet); per handle, so that handles of a multi-device handle, driven
                    //   by their own host threads, never share it
};
constexpr int kPersistForms = 8;  // (ICE, GATE, BOX) of the persistent band kernels

struct Chunk {
  int first;        // first window index (global)
  int count;
  int64_t base_n, base_m, base_nz;
};

// Launchers (dvh_kernels.hip).  Return hipError_t.
// list (nlist entries): global window indices, or null for the whole chunk.
hipError_t launch_setup(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n, int max_m,
                        hipStream_t s, const int32_t* list = nullptr, int nlist = 0);
// Solve kernel selection is made from the chunk maxima; returns hipErrorInvalidValue when no
// instantiation covers the sizes (the caller reports DVH_ERR_UNSUPPORTED).
// Generic (CSR) kernel; list = optional device list of window ids (nlist blocks) instead of the whole chunk.
hipError_t launch_pdhg(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n, int max_m,
                       int64_t max_nnz, hipStream_t s, int* variant_out, const int32_t* list, int nlist);
// ELL fast-path kernel over the whole chunk, or over the listed windows (wx, wy: ELL widths for K^T and K).
// Windows that do not fit its shape come back with istats status -1 (kNeedsGeneric) and must be re-run by
// launch_pdhg.
// latency: a list of at most two windows per CU (small variants only where they beat the 512-thread kernels).
hipError_t launch_pdhg_ell(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n, int max_m,
                           int wx, int wy, hipStream_t s, int* variant_out, const int32_t* list, int nlist,
                           bool latency = false);
// Battery-banded kernel (dvh_band.hip) over the whole chunk.  Windows whose CSR is not the battery + DCM
// window shape come back with istats status -2 (kNeedsEll) and must be re-run by launch_pdhg_ell.
// ice: the variant with LP-relaxed ICE columns (elec, on) and rows; list (nlist entries): global window indices,
// or null for the whole chunk; form: steps per lane of the battery kernel (3 default, 1 = the 768-thread form);
// variant_out: 9000000 + 1000 (steps per lane - 1) + 100 ice + waves per window.
// box (battery forms): iterate on the columns' [0, 1]-normalised boxes (dvh_band.hip, BOX); windows with an unbounded
// ch / dis / ene column come back with status -3 (kNeedsPlain) and must be re-run with box = false.
hipError_t launch_pdhg_band(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, hipStream_t s, bool ice,
                            int form, bool box, const int32_t* list, int nlist, int* variant_out);
// Its persistent forms (dvh_band_persist.hip), the default for the three-step battery form and the ICE form unless
// DVH_BAND_QUEUE=0 (DVH_BAND_QUEUE_ICE=0: the ICE form only); gate: dvh_options.kkt_predict > 0.
hipError_t launch_band_persist(bool gate, bool box, const Batch& b, const Work& w, const Chunk& ch, const Opts& o,
                               hipStream_t s, const int32_t* list, int nlist, int* variant_out);
hipError_t launch_band_persist_ice(bool gate, bool box, const Batch& b, const Work& w, const Chunk& ch, const Opts& o,
                                   hipStream_t s, const int32_t* list, int nlist, int* variant_out);
size_t setup_lds_bytes(int max_n, int max_m);
// Setup (scaling, transpose) of the listed medium windows (scaling vectors kept in the global workspace).
hipError_t launch_setup_medium(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int max_n,
                               const int32_t* list, int nlist, hipStream_t s);
// Medium tier (dvh_chain.hip): plan (structure check + segmentation, plan[kPlanInts] per listed window, plan[0] =
// P, 0 = not this tier, -1 = reported infeasible by the setup) and the team kernel over the windows at positions
// pos[] of the plan (PT workgroups per team, NT teams, cooperative launch; xbuf >= chain_xbuf_bytes(NT, PT)).
// The plan reads only the window's own (unscaled) data: it runs before the setup, reports crossed bounds itself
// (PRIMAL_INFEASIBLE, plan[0] = -1) and leaves the step -> DCM row / tau maps in the window's vbuf workspace.
hipError_t launch_chain_plan(const Batch& b, const Work& w, const Chunk& ch, const int32_t* list, int nlist,
                             int max_T, int32_t* plan, hipStream_t s);
// Grid-wide setup (scaling, scaled data, norms: what setup_kernel writes for the chain kernel) of one planned window
// whose n is too large for the one-workgroup setup; uses the plan's maps.
hipError_t launch_setup_long(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, int k, const int64_t* d,
                             hipStream_t s);
// istats status of the listed windows set to kChainPending before a team launch: after an aborted launch the windows
// still pending go to the grid-wide path
constexpr int kChainPending = -7;
hipError_t launch_chain_mark(const Batch& b, const int32_t* list, int nlist, hipStream_t s);
hipError_t chain_capacity(int device, int* blocks);
size_t chain_xbuf_bytes(int NT, int PT);
size_t chain_abort_bytes(int S);  // abort word, window counter, per-workgroup diagnostics (grid 8 S)
// S: resident workgroup slots per XCD (grid = 8 S); teams of PT workgroups, chain_team_count(S, PT) of them
int chain_team_count(int S, int PT);
// spin_ticks: the longest a segment waits for a partner's exchange (wall-clock ticks) before the launch aborts
hipError_t launch_chain(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, const int32_t* pos, int npos,
                        const int32_t* plan, int PT, int S, void* xbuf, int32_t* abort_word, long long spin_ticks,
                        hipStream_t s);
// Seeded-sweep warm starts (dvh_sweep.hip): rows[count][q + 2] = {window, partner windows (q), T (> 0: battery + DCM
// dual scaling)}, wts[count][q] the partners' weights; bad counts rows whose windows differ in shape (skipped).
constexpr int kMaxBlend = 8;  // partners per window
hipError_t launch_warm_transfer(const int64_t* desc, const double* c, const double* u, double* x, double* y,
                                const int32_t* rows, const double* wts, int q, int count, int32_t* bad, hipStream_t s);
// Synthetic scenario series (dvh_series.hip): numpy-identical draws, one thread per scenario (ambiguous counts
// scenarios with a wedge test too close to call), and the device builder's inputs of G windows (bad counts rows out of
// range).
hipError_t launch_series_draws(const uint64_t* seeds, int count, int steps, int n_unif, double a1, double innov,
                               double* z0, double* ar, double* unif, int32_t* ambiguous, int32_t* amb_rows,
                               hipStream_t s);
hipError_t launch_series_windows(const ::dvh_window_series& w, int32_t* bad, hipStream_t s);
// Cascade lists on the device (dvh_route.hip): the small windows of [first, first + count) -- or of in_list[0 ..
// count) -- whose status is `want` (cls 1: and n <= lim_n, m <= lim_m; cls 2: the others; cls 0: any size), in order,
// to out_list; out_info[0..5] = {their number, max ELL widths wx, wy, max n, m, nnz} over them.
hipError_t launch_route(const int64_t* desc, const int32_t* istats, const double* scal, int first, int count,
                        const int32_t* in_list, int want, int small_max, int cls, int lim_n, int lim_m,
                        int32_t* out_list, int32_t* out_info, hipStream_t s);
// Power iteration for ||Kt||_2 of the listed windows (generic path; the ELL kernel does its own on chip).
hipError_t launch_power(const Batch& b, const Work& w, const Chunk& ch, const Opts& o, const int32_t* list, int nlist,
                        hipStream_t s);

// Post-facto reliability sweep (dvh_outage.hip): one case of dvh_outage_case with device pointers.
struct OutageCase {
  int n_steps, max_steps, outage_len, pad;
  int64_t len_off, hist_off;  // offsets into the lengths / histogram outputs
  double dt, soe0, dg_gen, gamma, soe_min, soe_max, charge_max, discharge_max, rte;
  const double *critical_load, *pv_max, *pv_vari, *init_soe, *load_shed;
};
// One thread per (case, start step); hist must be zeroed (sum of outage_len + 1 bins); lengths may be null.
hipError_t launch_outage(const OutageCase* d_cases, int ncase, int max_steps_n, int max_bins, int32_t* d_lengths,
                         int32_t* d_hist, hipStream_t s);
// min_soe_iterative mode: soe_used (max - min SOE of a target-length outage from soe0) per start.
hipError_t launch_outage_min_soe(const OutageCase* d_cases, int ncase, int max_steps_n, double* d_soe_used,
                                 hipStream_t s);

// Grid-wide PDHG for one window too large for the workgroup-per-window kernels (dvh_large.hip).
struct LargeSolver;
LargeSolver* large_create();
void large_destroy(LargeSolver* ls);

// The result all-gather's RCCL communicator (dvh_comm.cpp; dvh_comm_init / dvh_gather_results).  Return codes are the
// DVH_* codes; messages go to *err.
constexpr int kCommIdBytes = 128;  // ncclUniqueId
struct Comm;
int comm_unique_id(unsigned char* id, std::string* err);
int comm_init(int device, int rank, int world, const unsigned char* id, Comm** out, std::string* err);
int comm_all_gather(Comm* c, const void* send, void* recv, size_t bytes, hipStream_t s, std::string* err);
void comm_info(const Comm* c, int* rank, int* world);
void comm_destroy(Comm* c);
// Solves window k (desc row d) of the batch on stream s; writes b.x / b.y / b.stats / b.istats of window k.
hipError_t large_solve(LargeSolver* ls, const Batch& b, int k, const int64_t* d, const Opts& o, const double* hinv,
                       hipStream_t s, std::string* err, float* setup_ms, float* pdhg_ms);

}  // namespace dvh

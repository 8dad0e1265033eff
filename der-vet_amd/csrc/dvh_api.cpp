// dvh_api.cpp -- C ABI of libdervet_hip (declared in include/dervet_hip.h).
//
// Replaces the per-window solve of storagevet Scenario.solve_optimization (dervet/MicrogridScenario.py:319)
// for a whole batch of windows: validates and packs host LPs, moves them to HBM, runs the setup and PDHG
// kernels chunk by chunk on the handle's stream, and copies primal/dual solutions and statistics back.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dervet_hip.h"
#include "dvh_internal.h"
#include "dvh_validate.h"

#define DVH_VERSION_STRING "dervet_hip 0.1.0 (gfx950, restarted reflected-Halpern PDHG)"

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t want) {
    if (want <= bytes) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
    want = std::max<size_t>(want, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) bytes = want;
    return e;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

constexpr int kChunkWindows = 262144;

}  // namespace

struct dvh_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  dvh_options opts{};
  std::string err;
  // packed inputs / outputs for the host API
  DevBuf d_desc, d_indptr, d_indices, d_data, d_c, d_c0, d_q, d_l, d_u, d_x, d_y, d_stats, d_istats;
  // workspace
  DevBuf w_queue;  // the band kernels' work-queue counter
  int band_slots[dvh::kPersistForms] = {};  // the persistent band forms' resident slots on this device (Work::slots)
  DevBuf w_tptr, w_tind, w_tval, w_kval, w_rowof, w_perm, w_dr, w_dc, w_cs, w_ls, w_us, w_qs, w_vbuf, w_wbuf,
      w_tmpc, w_tmpr, w_longk, w_longt, w_scal, w_fc, w_fr;
  DevBuf d_list, d_hinv;
  DevBuf m_list, m_plan, m_pos, m_xbuf, m_abort;  // medium tier (dvh_chain.hip)
  int chain_cap = -1;                             // resident 768-thread workgroups (cooperative limit)
  long long spin_ticks = 0;                       // chain kernel: longest exchange wait (wall-clock ticks)
  int n_chain_aborts = 0;                         // team launches of the last solve that aborted (unfinished windows
                                                  // ran grid-wide); dvh_last_chain_aborts
  std::string warn;                               // diagnostics of the last solve's fallbacks (dvh_last_warning)
  DevBuf o_data, o_cases, o_len, o_hist, o_soe;  // reliability sweep
  DevBuf s_pairs, s_wts, s_bad;                   // seeded-sweep warm transfer (dvh_sweep.hip)
  DevBuf g_seeds, g_word;                         // scenario series generator (dvh_series.hip)
  DevBuf d_route;                                 // cascade lists' counts / ELL widths (dvh_route.hip)
  int32_t* route_host = nullptr;                  // their pinned host mirror (one small read-back per tier)
  int n_syncs = 0;                                // host waits on the stream in the last solve
  double outage_ms = 0.0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // per-chunk timing events: a pool created on first use and reused by every solve (destroyed with the handle), so
  // no exit path of a solve can leak them; chunk_used = the events of the last solve
  std::vector<std::array<hipEvent_t, 3>> chunk_events;
  size_t chunk_used = 0;
  double timing[3] = {0, 0, 0};
  int last_variant = -1;
  int n_ell = 0, n_generic = 0, n_large = 0, n_band = 0, n_chain = 0;
  int kernel_path = 0;  // 0 band -> ELL -> generic, 1 generic only, 2 ELL -> generic (no band kernel), 3 / 4 as 0
                        // with the battery band kernel's one-step / three-step form forced (0 picks by batch size)
  int cus = 0;          // compute units of the device (band kernel form choice)
  std::vector<int32_t> order;  // dvh_set_launch_order: the next solve's band-pass window order (empty: packing order)
  std::vector<int32_t> order_used;  // (the copy a solve consumed: kept until the next one, the H2D copy reads it)
  DevBuf d_order;
  dvh::LargeSolver* large = nullptr;  // grid-wide path for windows above dvh::kSmallMax (created on first use)
  float large_ms[2] = {0, 0};         // setup, PDHG time of the large windows of the last solve
  // Further devices of this handle (device_mask bits after the first, or dvh_create_devices): same options; a
  // host-buffer batch is split into contiguous, cost-balanced ranges, one per device, solved concurrently (one host
  // thread per device, no inter-device traffic), results written straight into the caller's buffers.
  std::vector<dvh_handle*> peers;
  dvh::Comm* comm = nullptr;  // dvh_comm_init: the result all-gather's RCCL communicator (dvh_comm.cpp)
};

// Every host wait on a solve's stream goes through here (dvh_last_host_syncs reports the count of the last solve).
static hipError_t sync_stream(dvh_handle* h, hipStream_t s) {
  ++h->n_syncs;
  return hipStreamSynchronize(s);
}

static int fail(dvh_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  return code;
}

static int hip_fail(dvh_handle* h, hipError_t e, const char* where) {
  return fail(h, DVH_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define DVH_HIP(h, call)                                 \
  do {                                                   \
    hipError_t e_ = (call);                              \
    if (e_ != hipSuccess) return hip_fail(h, e_, #call); \
  } while (0)

extern "C" {

const char* dvh_version(void) { return DVH_VERSION_STRING; }

void dvh_default_options(dvh_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->eps = 1e-6;
  o->max_iters = 100000;
  o->check_every = 32;
  o->kkt_every = 4;
  o->ruiz_iters = 10;
  o->power_iters = 64;
  o->step_safety = 0.998;
  o->reflection = 1.0;
  o->restart_sufficient = 0.2;
  o->restart_necessary = 0.8;
  o->restart_artificial = 0.1;
  o->primal_weight_theta = 1.0;
  o->verbose = 0;
  o->eps_obj = 1e-6;
}

static std::string check_options(const dvh_options* o) {
  if (!(o->eps > 0.0)) return "eps must be > 0";
  if (!(o->eps_obj >= 0.0)) return "eps_obj must be >= 0";
  if (o->max_iters <= 0) return "max_iters must be > 0";
  if (o->check_every <= 0) return "check_every must be > 0";
  if (o->kkt_every <= 0) return "kkt_every must be > 0";
  if (o->kkt_predict < 0) return "kkt_predict must be >= 0";
  if (o->ruiz_iters < 0 || o->power_iters <= 0) return "ruiz_iters must be >= 0 and power_iters > 0";
  if (!(o->step_safety > 0.0 && o->step_safety < 1.0)) return "step_safety must be in (0, 1)";
  if (!(o->reflection >= 0.0 && o->reflection <= 1.0)) return "reflection must be in [0, 1]";
  return "";
}

static int create_one(int dev, const dvh_options* opts, dvh_handle** out);

int dvh_create_devices(const int32_t* devices, int32_t n, const dvh_options* opts, dvh_handle** out) {
  if (!out || !devices || n < 1) return DVH_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return DVH_ERR_HIP;
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= ndev) return DVH_ERR_ARG;
  dvh_handle* h = nullptr;
  if (int rc = create_one(devices[0], opts, &h)) return rc;
  for (int i = 1; i < n; ++i) {
    dvh_handle* p = nullptr;
    if (int rc = create_one(devices[i], opts, &p)) {
      dvh_destroy(h);
      return rc;
    }
    h->peers.push_back(p);
  }
  *out = h;
  return DVH_OK;
}

int dvh_create(int device_mask, const dvh_options* opts, dvh_handle** out) {
  if (!out) return DVH_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return DVH_ERR_HIP;
  std::vector<int32_t> devs;
  for (int d = 0; d < 31 && d < ndev; ++d)
    if ((device_mask >> d) & 1) devs.push_back(d);
  if (device_mask <= 0) devs = {0};
  if (devs.empty() || (device_mask >> std::min(ndev, 31)) != 0) return DVH_ERR_ARG;  // a bit beyond the devices
  return dvh_create_devices(devs.data(), (int32_t)devs.size(), opts, out);
}

static int create_one(int dev, const dvh_options* opts, dvh_handle** out) {
  dvh_handle* h = new dvh_handle();
  h->device = dev;
  dvh_default_options(&h->opts);
  if (opts) {
    std::string m = check_options(opts);
    if (!m.empty()) {
      delete h;
      return DVH_ERR_ARG;
    }
    h->opts = *opts;
  }
  if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return DVH_ERR_HIP;
  }
  for (auto& e : h->ev) hipEventCreate(&e);
  {  // Halpern weight table 1/(k+2): exact IEEE quotients, identical to the host restatement
    std::vector<double> tab(dvh::kHalpernTab);
    for (int k = 0; k < dvh::kHalpernTab; ++k) tab[k] = 1.0 / (k + 2.0);
    if (h->d_hinv.ensure(sizeof(double) * tab.size()) != hipSuccess ||
        hipMemcpy(h->d_hinv.p, tab.data(), sizeof(double) * tab.size(), hipMemcpyHostToDevice) != hipSuccess) {
      dvh_destroy(h);
      return DVH_ERR_HIP;
    }
  }
  *out = h;
  return DVH_OK;
}

int dvh_set_options(dvh_handle* h, const dvh_options* opts) {
  if (!h || !opts) return DVH_ERR_ARG;
  std::string m = check_options(opts);
  if (!m.empty()) return fail(h, DVH_ERR_ARG, m);
  h->opts = *opts;
  for (dvh_handle* p : h->peers) p->opts = *opts;
  return DVH_OK;
}

int dvh_device_count(const dvh_handle* h) { return h ? 1 + (int)h->peers.size() : 0; }

int dvh_destroy(dvh_handle* h) {
  if (!h) return DVH_ERR_ARG;
  for (dvh_handle* p : h->peers) dvh_destroy(p);
  h->peers.clear();
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  DevBuf* bufs[] = {&h->d_desc, &h->d_indptr, &h->d_indices, &h->d_data, &h->d_c, &h->d_c0, &h->d_q, &h->d_l,
                    &h->d_u, &h->d_list, &h->d_hinv, &h->d_x, &h->d_y, &h->d_stats, &h->d_istats, &h->w_tptr, &h->w_tind, &h->w_tval,
                    &h->w_kval, &h->w_rowof, &h->w_perm, &h->w_dr, &h->w_dc, &h->w_cs, &h->w_ls, &h->w_us,
                    &h->w_qs, &h->w_vbuf, &h->w_wbuf, &h->w_tmpc, &h->w_tmpr, &h->w_longk, &h->w_longt, &h->w_scal,
                    &h->w_fc, &h->w_fr,
                    &h->m_list, &h->m_plan, &h->m_pos, &h->m_xbuf, &h->m_abort, &h->o_data, &h->o_cases, &h->o_len, &h->o_hist, &h->o_soe,
                    &h->s_pairs, &h->s_wts, &h->s_bad, &h->g_seeds, &h->g_word, &h->d_route, &h->d_order, &h->w_queue};
  for (DevBuf* b : bufs) b->release();
  if (h->route_host) hipHostFree(h->route_host);
  for (auto& e : h->ev)
    if (e) hipEventDestroy(e);
  for (auto& ce : h->chunk_events)
    for (hipEvent_t e : ce)
      if (e) hipEventDestroy(e);
  h->chunk_events.clear();
  if (h->large) dvh::large_destroy(h->large);
  if (h->comm) dvh::comm_destroy(h->comm);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return DVH_OK;
}

const char* dvh_last_error(const dvh_handle* h) { return h ? h->err.c_str() : "null handle"; }

// ---- the result all-gather across ranks (dvh_comm.cpp)
int dvh_comm_unique_id(dvh_handle* h, uint8_t* id) {
  if (!h || !id) return DVH_ERR_ARG;
  return dvh::comm_unique_id(id, &h->err);
}

int dvh_comm_init(dvh_handle* h, int32_t rank, int32_t world, const uint8_t* id) {
  if (!h || !id || world < 1 || rank < 0 || rank >= world) return fail(h, DVH_ERR_ARG, "dvh_comm_init: rank / world");
  if (!h->peers.empty())
    return fail(h, DVH_ERR_ARG, "dvh_comm_init: one communicator rank per device; this handle spans several");
  if (h->comm) return fail(h, DVH_ERR_ARG, "dvh_comm_init: the handle already has a communicator");
  return dvh::comm_init(h->device, rank, world, id, &h->comm, &h->err);
}

int dvh_comm_info(const dvh_handle* h, int32_t* rank_world) {
  if (!h || !rank_world) return DVH_ERR_ARG;
  if (!h->comm) {
    rank_world[0] = 0;
    rank_world[1] = 0;
    return DVH_OK;
  }
  int r = 0, w = 0;
  dvh::comm_info(h->comm, &r, &w);
  rank_world[0] = r;
  rank_world[1] = w;
  return DVH_OK;
}

int dvh_gather_results(dvh_handle* h, const void* rows, uint64_t bytes_per_rank, void* out, void* stream) {
  if (!h || !rows || !out) return DVH_ERR_ARG;
  if (!h->comm) return fail(h, DVH_ERR_ARG, "dvh_gather_results: no communicator (dvh_comm_init)");
  if (bytes_per_rank == 0) return DVH_OK;
  hipSetDevice(h->device);
  hipStream_t s = stream ? (hipStream_t)stream : h->stream;
  return dvh::comm_all_gather(h->comm, rows, out, (size_t)bytes_per_rank, s, &h->err);
}
const char* dvh_last_warning(const dvh_handle* h) { return h ? h->warn.c_str() : "null handle"; }

int dvh_warm_transfer_blend(dvh_handle* h, const dvh_packed* b, const int32_t* rows, const double* weights,
                            int32_t count, int32_t q) {
  if (!h) return DVH_ERR_ARG;
  if (q < 1 || q > dvh::kMaxBlend) return fail(h, DVH_ERR_ARG, "warm transfer: partners per window must be 1..8");
  if (count < 0 || (count > 0 && (!b || !rows || !weights))) return fail(h, DVH_ERR_ARG, "warm transfer: bad arguments");
  if (count == 0) return DVH_OK;
  if (!b->desc || !b->c || !b->u || !b->x || !b->y) return fail(h, DVH_ERR_ARG, "null device array in packed batch");
  const size_t R = (size_t)q + 2;
  // every window written once, no partner written (a workgroup would read it while another writes it), finite weights
  std::vector<char> target((size_t)std::max(b->count, 0), 0);
  for (int32_t i = 0; i < count; ++i) {
    const int32_t w = rows[R * i];
    if (w < 0 || w >= b->count)
      return fail(h, DVH_ERR_ARG, "warm transfer: row " + std::to_string(i) + " names no window");
    for (int32_t k = 0; k < q; ++k) {
      const int32_t p = rows[R * i + 1 + k];
      if (p < 0 || p >= b->count || w == p)
        return fail(h, DVH_ERR_ARG, "warm transfer: pair " + std::to_string(i) + " names no window / itself");
      if (!std::isfinite(weights[(size_t)q * i + k]))
        return fail(h, DVH_ERR_ARG, "warm transfer: weight of row " + std::to_string(i) + " is not finite");
    }
    if (target[w]) return fail(h, DVH_ERR_ARG, "warm transfer: window " + std::to_string(w) + " listed twice");
    target[w] = 1;
  }
  for (int32_t i = 0; i < count; ++i)
    for (int32_t k = 0; k < q; ++k)
      if (target[rows[R * i + 1 + k]])
        return fail(h, DVH_ERR_ARG, "warm transfer: partner of pair " + std::to_string(i) + " is itself a listed window");
  DVH_HIP(h, hipSetDevice(h->device));
  hipStream_t s = h->stream;
  DVH_HIP(h, h->s_pairs.ensure(sizeof(int32_t) * R * (size_t)count));
  DVH_HIP(h, h->s_wts.ensure(sizeof(double) * (size_t)q * (size_t)count));
  DVH_HIP(h, h->s_bad.ensure(sizeof(int32_t)));
  DVH_HIP(h, hipMemcpyAsync(h->s_pairs.p, rows, sizeof(int32_t) * R * (size_t)count, hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipMemcpyAsync(h->s_wts.p, weights, sizeof(double) * (size_t)q * (size_t)count, hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipMemsetAsync(h->s_bad.p, 0, sizeof(int32_t), s));
  hipError_t e = dvh::launch_warm_transfer(b->desc, b->c, b->u, b->x, b->y, h->s_pairs.as<int32_t>(),
                                           h->s_wts.as<double>(), q, count, h->s_bad.as<int32_t>(), s);
  if (e != hipSuccess) return hip_fail(h, e, "launch_warm_transfer");
  int32_t bad = 0;
  DVH_HIP(h, hipMemcpyAsync(&bad, h->s_bad.p, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  DVH_HIP(h, hipStreamSynchronize(s));
  if (bad) return fail(h, DVH_ERR_ARG, "warm transfer: " + std::to_string(bad) + " pair(s) of different LP shape");
  return DVH_OK;
}

int dvh_warm_transfer(dvh_handle* h, const dvh_packed* b, const int32_t* pairs, int32_t count) {
  if (!h) return DVH_ERR_ARG;
  if (count < 0 || (count > 0 && (!b || !pairs))) return fail(h, DVH_ERR_ARG, "warm transfer: bad arguments");
  const std::vector<double> ones((size_t)std::max(count, 0), 1.0);  // one partner, weight 1: the plain transfer
  return dvh_warm_transfer_blend(h, b, pairs, ones.data(), count, 1);
}

int dvh_series_draws(dvh_handle* h, const dvh_sweep_draws* d) {
  if (!h) return DVH_ERR_ARG;
  if (!d || d->count < 0 || d->steps < 1 || d->n_uniform < 0)
    return fail(h, DVH_ERR_ARG, "series draws: bad sizes");
  if (d->count == 0) return DVH_OK;
  if (!d->seeds || !d->z0 || !d->ar || (d->n_uniform > 0 && !d->uniform))
    return fail(h, DVH_ERR_ARG, "series draws: null array");
  DVH_HIP(h, hipSetDevice(h->device));
  hipStream_t s = h->stream;
  DVH_HIP(h, h->g_seeds.ensure(sizeof(uint64_t) * (size_t)d->count));
  DVH_HIP(h, h->g_word.ensure(sizeof(int32_t)));
  DVH_HIP(h, hipMemcpyAsync(h->g_seeds.p, d->seeds, sizeof(uint64_t) * (size_t)d->count, hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipMemsetAsync(h->g_word.p, 0, sizeof(int32_t), s));
  hipError_t e = dvh::launch_series_draws(h->g_seeds.as<uint64_t>(), d->count, d->steps, d->n_uniform, d->a1,
                                          d->innov, d->z0, d->ar, d->uniform, h->g_word.as<int32_t>(), d->ambiguous,
                                          s);
  if (e != hipSuccess) return hip_fail(h, e, "launch_series_draws");
  int32_t amb = 0;
  DVH_HIP(h, hipMemcpyAsync(&amb, h->g_word.p, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  DVH_HIP(h, hipStreamSynchronize(s));
  if (amb && !d->ambiguous)
    return fail(h, DVH_ERR_UNSUPPORTED, "series draws: " + std::to_string(amb) +
                                            " scenario(s) met a ziggurat wedge test within 2^-40 of exp(); their "
                                            "draws may differ from numpy's");
  return DVH_OK;
}

int dvh_series_windows(dvh_handle* h, const dvh_window_series* w) {
  if (!h) return DVH_ERR_ARG;
  if (!w || w->G < 0 || w->T < 1 || w->t0 < 0 || w->rep < 1 || w->J < 0 || w->count < 1 || w->hours < 1 ||
      !(w->dt > 0.0) || (int64_t)(w->t0 + w->T - 1) / w->rep >= w->hours)
    return fail(h, DVH_ERR_ARG, "series windows: bad sizes (window past the series?)");
  if (w->G == 0) return DVH_OK;
  if (!w->rows || !w->ar || !w->site_load || !w->pv_profile || !w->price || !w->load_scale || !w->price_scale ||
      !w->pv_rated || !w->hp || !w->c0_add || !w->base || !w->retail || !w->c0)
    return fail(h, DVH_ERR_ARG, "series windows: null array");
  DVH_HIP(h, hipSetDevice(h->device));
  hipStream_t s = h->stream;
  DVH_HIP(h, h->g_word.ensure(sizeof(int32_t)));
  DVH_HIP(h, hipMemsetAsync(h->g_word.p, 0, sizeof(int32_t), s));
  hipError_t e = dvh::launch_series_windows(*w, h->g_word.as<int32_t>(), s);
  if (e != hipSuccess) return hip_fail(h, e, "launch_series_windows");
  int32_t bad = 0;
  DVH_HIP(h, hipMemcpyAsync(&bad, h->g_word.p, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  DVH_HIP(h, hipStreamSynchronize(s));
  if (bad) return fail(h, DVH_ERR_ARG, "series windows: " + std::to_string(bad) + " row(s) outside 0 .. count - 1");
  return DVH_OK;
}

int dvh_synchronize(dvh_handle* h) {
  if (!h) return DVH_ERR_ARG;
  DVH_HIP(h, hipStreamSynchronize(h->stream));
  return DVH_OK;
}

int dvh_last_host_syncs(const dvh_handle* h, int32_t* out) {
  if (!h || !out) return DVH_ERR_ARG;
  *out = h->n_syncs;
  return DVH_OK;
}

int dvh_last_stats(const dvh_handle* h, int32_t* out4) {
  if (!h || !out4) return DVH_ERR_ARG;
  out4[0] = h->n_ell;
  out4[1] = h->n_generic;
  out4[2] = h->last_variant;
  out4[3] = h->kernel_path == 1 ? 1 : 0;
  return DVH_OK;
}

int dvh_last_path_counts(const dvh_handle* h, int32_t* out3) {
  if (!h || !out3) return DVH_ERR_ARG;
  out3[0] = h->n_ell;
  out3[1] = h->n_generic;
  out3[2] = h->n_large;
  return DVH_OK;
}

int dvh_last_chain_aborts(const dvh_handle* h, int32_t* out) {
  if (!h || !out) return DVH_ERR_ARG;
  *out = h->n_chain_aborts;
  return DVH_OK;
}

int dvh_last_path_counts5(const dvh_handle* h, int32_t* out5) {
  if (!h || !out5) return DVH_ERR_ARG;
  out5[0] = h->n_ell;
  out5[1] = h->n_generic;
  out5[2] = h->n_large;
  out5[3] = h->n_band;
  out5[4] = h->n_chain;
  return DVH_OK;
}

int dvh_last_path_counts4(const dvh_handle* h, int32_t* out4) {
  if (!h || !out4) return DVH_ERR_ARG;
  out4[0] = h->n_ell;
  out4[1] = h->n_generic;
  out4[2] = h->n_large;
  out4[3] = h->n_band;
  return DVH_OK;
}

int dvh_set_launch_order(dvh_handle* h, const int32_t* order, int32_t count) {
  if (!h || count < 0 || (count > 0 && !order)) return DVH_ERR_ARG;
  h->order.clear();
  if (count == 0) return DVH_OK;
  std::vector<char> seen(count, 0);  // a permutation of 0 .. count - 1 (the kernels index windows with it)
  for (int32_t i = 0; i < count; ++i) {
    const int32_t k = order[i];
    if (k < 0 || k >= count || seen[k]) return fail(h, DVH_ERR_ARG, "launch order is not a permutation of 0 .. count - 1");
    seen[k] = 1;
  }
  h->order.assign(order, order + count);
  return DVH_OK;
}

int dvh_set_kernel_path(dvh_handle* h, int mode) {
  if (!h || mode < 0 || mode > 4) return DVH_ERR_ARG;
  h->kernel_path = mode;
  for (dvh_handle* p : h->peers) p->kernel_path = mode;
  return DVH_OK;
}

// Validates the outage cases and moves them to the device (o_data / o_cases); olen[k] = simulated outage steps
// (int(max_outage / dt), or int(target_hours[k] / dt) for the min-SOE mode).
struct OutagePack {
  std::vector<int> olen;
  size_t nlen = 0, nhist = 0;
  int max_n = 0, max_bins = 0;
};
static int outage_pack(dvh_handle* h, const dvh_outage_case* cases, int32_t count, const int32_t* target_hours,
                       OutagePack& P) {
  hipSetDevice(h->device);
  size_t nd = 0, nlen = 0, nhist = 0;
  int max_n = 0, max_bins = 0;
  std::vector<int>& olen = P.olen;
  olen.assign(count, 0);
  for (int k = 0; k < count; ++k) {
    const dvh_outage_case& c = cases[k];
    const std::string w = "outage case " + std::to_string(k) + ": ";
    if (c.n_steps < 1 || !c.critical_load) return fail(h, DVH_ERR_ARG, w + "n_steps >= 1 and critical_load required");
    if (!(c.dt > 0.0) || c.max_outage < 1 || c.max_outage / c.dt < 1.0)
      return fail(h, DVH_ERR_ARG, w + "dt > 0 and max_outage >= dt required");
    if (!(c.rte > 0.0)) return fail(h, DVH_ERR_ARG, w + "rte must be > 0");
    olen[k] = (int)(c.max_outage / c.dt);  // int(self.max_outage_duration / self.dt), Reliability.py:917
    if (target_hours) {  // outage_len = self.outage_duration / self.dt (min_soe_iterative, :712)
      if (target_hours[k] < 1 || target_hours[k] / c.dt < 1.0)
        return fail(h, DVH_ERR_ARG, w + "target outage hours must be >= dt");
      olen[k] = (int)(target_hours[k] / c.dt);
    }
    if (olen[k] + 1 > 16384) return fail(h, DVH_ERR_UNSUPPORTED, w + "more than 16384 outage steps");
    nd += (size_t)c.n_steps * (1 + (c.pv_max ? 1 : 0) + (c.pv_vari ? 1 : 0) + (c.init_soe ? 1 : 0)) +
          (c.load_shed_pct ? (size_t)c.max_outage : 0);
    nlen += (size_t)c.n_steps;
    nhist += (size_t)olen[k] + 1;
    max_n = std::max(max_n, c.n_steps);
    max_bins = std::max(max_bins, olen[k] + 1);
  }
  std::vector<double> data(std::max<size_t>(nd, 1));
  std::vector<dvh::OutageCase> dc(count);
  DVH_HIP(h, h->o_data.ensure(sizeof(double) * data.size()));
  DVH_HIP(h, h->o_cases.ensure(sizeof(dvh::OutageCase) * count));
  DVH_HIP(h, h->o_len.ensure(sizeof(int32_t) * nlen));
  DVH_HIP(h, h->o_hist.ensure(sizeof(int32_t) * nhist));
  const double* dbase = h->o_data.as<double>();
  size_t off = 0, lo = 0, ho = 0;
  auto put = [&](const double* src, size_t n) -> const double* {
    if (!src) return nullptr;
    std::memcpy(&data[off], src, sizeof(double) * n);
    const double* d = dbase + off;
    off += n;
    return d;
  };
  for (int k = 0; k < count; ++k) {
    const dvh_outage_case& c = cases[k];
    dvh::OutageCase& o = dc[k];
    o.n_steps = c.n_steps;
    o.max_steps = c.max_outage;
    o.outage_len = olen[k];
    o.pad = 0;
    o.len_off = (int64_t)lo;
    o.hist_off = (int64_t)ho;
    o.dt = c.dt;
    o.soe0 = c.soe0;
    o.dg_gen = c.dg_gen;
    o.gamma = c.gamma;
    o.soe_min = c.soe_min;
    o.soe_max = c.soe_max;
    o.charge_max = c.charge_max;
    o.discharge_max = c.discharge_max;
    o.rte = c.rte;
    o.critical_load = put(c.critical_load, c.n_steps);
    o.pv_max = put(c.pv_max, c.n_steps);
    o.pv_vari = put(c.pv_vari, c.n_steps);
    o.init_soe = put(c.init_soe, c.n_steps);
    o.load_shed = put(c.load_shed_pct, c.max_outage);
    lo += c.n_steps;
    ho += olen[k] + 1;
  }
  hipStream_t s = h->stream;
  DVH_HIP(h, hipMemcpyAsync(h->o_data.p, data.data(), sizeof(double) * data.size(), hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipMemcpyAsync(h->o_cases.p, dc.data(), sizeof(dvh::OutageCase) * count, hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipStreamSynchronize(s));  // the host staging vectors end here
  P.nlen = nlen;
  P.nhist = nhist;
  P.max_n = max_n;
  P.max_bins = max_bins;
  return DVH_OK;
}

int dvh_outage_coverage(dvh_handle* h, const dvh_outage_case* cases, int32_t count, int32_t* lengths,
                        double* lcp) {
  if (!h) return DVH_ERR_ARG;
  if (count < 0 || (count > 0 && (!cases || !lcp))) return fail(h, DVH_ERR_ARG, "cases and lcp are required");
  if (count == 0) return DVH_OK;
  OutagePack P;
  if (int rc = outage_pack(h, cases, count, nullptr, P)) return rc;
  const std::vector<int>& olen = P.olen;
  const size_t nlen = P.nlen, nhist = P.nhist;
  const int max_n = P.max_n, max_bins = P.max_bins;
  hipStream_t s = h->stream;
  DVH_HIP(h, hipMemsetAsync(h->o_hist.p, 0, sizeof(int32_t) * nhist, s));
  DVH_HIP(h, hipEventRecord(h->ev[0], s));
  hipError_t e = dvh::launch_outage(h->o_cases.as<dvh::OutageCase>(), count, max_n, max_bins,
                                    lengths ? h->o_len.as<int32_t>() : nullptr, h->o_hist.as<int32_t>(), s);
  if (e != hipSuccess) return hip_fail(h, e, "launch_outage");
  DVH_HIP(h, hipEventRecord(h->ev[3], s));
  std::vector<int32_t> hist(nhist);
  DVH_HIP(h, hipMemcpyAsync(hist.data(), h->o_hist.p, sizeof(int32_t) * nhist, hipMemcpyDeviceToHost, s));
  if (lengths) DVH_HIP(h, hipMemcpyAsync(lengths, h->o_len.p, sizeof(int32_t) * nlen, hipMemcpyDeviceToHost, s));
  DVH_HIP(h, hipStreamSynchronize(s));
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, h->ev[0], h->ev[3]) == hipSuccess) h->outage_ms = ms;
  // the curve, in the reference's float64 arithmetic (Reliability.py:947-957)
  size_t po = 0, ho = 0;
  for (int k = 0; k < count; ++k) {
    const dvh_outage_case& c = cases[k];
    double length = c.dt;
    int j = 0;
    while (length <= (double)c.max_outage && j < olen[k]) {
      const int first = (int)(length / c.dt);
      double covered = 0.0;
      for (int b = first; b <= olen[k]; ++b) covered += (double)hist[ho + b];
      const double total = (double)c.n_steps - (length / c.dt) + 1.0;
      lcp[po + j] = covered / total;
      ++j;
      length += c.dt;
    }
    for (; j < olen[k]; ++j) lcp[po + j] = NAN;
    po += olen[k];
    ho += olen[k] + 1;
  }
  return DVH_OK;
}

int dvh_outage_min_soe(dvh_handle* h, const dvh_outage_case* cases, int32_t count, const int32_t* target_hours,
                       double* min_soe) {
  if (!h) return DVH_ERR_ARG;
  if (count < 0 || (count > 0 && (!cases || !target_hours || !min_soe)))
    return fail(h, DVH_ERR_ARG, "cases, target_hours and min_soe are required");
  if (count == 0) return DVH_OK;
  OutagePack P;
  if (int rc = outage_pack(h, cases, count, target_hours, P)) return rc;
  hipStream_t s = h->stream;
  DVH_HIP(h, h->o_soe.ensure(sizeof(double) * P.nlen));
  DVH_HIP(h, hipEventRecord(h->ev[0], s));
  hipError_t e = dvh::launch_outage_min_soe(h->o_cases.as<dvh::OutageCase>(), count, P.max_n, h->o_soe.as<double>(), s);
  if (e != hipSuccess) return hip_fail(h, e, "launch_outage_min_soe");
  DVH_HIP(h, hipEventRecord(h->ev[3], s));
  DVH_HIP(h, hipMemcpyAsync(min_soe, h->o_soe.p, sizeof(double) * P.nlen, hipMemcpyDeviceToHost, s));
  DVH_HIP(h, hipStreamSynchronize(s));
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, h->ev[0], h->ev[3]) == hipSuccess) h->outage_ms = ms;
  return DVH_OK;
}

int dvh_last_outage_ms(const dvh_handle* h, double* ms) {
  if (!h || !ms) return DVH_ERR_ARG;
  *ms = h->outage_ms;
  return DVH_OK;
}

int dvh_last_timing(const dvh_handle* h, double* ms3) {
  if (!h || !ms3) return DVH_ERR_ARG;
  for (int i = 0; i < 3; ++i) ms3[i] = h->timing[i];
  return DVH_OK;
}

}  // extern "C"

namespace dvh {
hipError_t launch_build_battery(const dvh_battery_group& g, const dvh_packed& b, int first, hipStream_t s);
}

extern "C" int dvh_build_battery_group(dvh_handle* h, const dvh_battery_group* g, const dvh_packed* b,
                                       int32_t first) {
  if (!h) return DVH_ERR_ARG;
  if (!g || !b) return fail(h, DVH_ERR_ARG, "null group or batch");
  if (g->G == 0) return DVH_OK;
  if (g->T < 1 || g->J < 0 || g->G < 0 || g->mI < 0 || !(g->dt > 0.0) || first < 0 || first + g->G > b->count)
    return fail(h, DVH_ERR_ARG, "battery group: bad sizes or window range");
  if ((g->mI > 0 && (!g->dcm_t || !g->dcm_j)) || !g->base || (g->J > 0 && !g->demand) || !g->E || !g->pch ||
      !g->pdis || !g->rte || !g->sdr || !g->soc_target || !g->ulsoc || !g->llsoc || !g->om || !g->c0 ||
      (g->has_retail && !g->retail) || (g->has_da && !g->da) || (g->has_emin && !g->emin) ||
      (g->has_emax && !g->emax) || (g->has_ice && (!g->ice_cap || !g->ice_pmin || !g->ice_cost)))
    return fail(h, DVH_ERR_ARG, "battery group: null input array");
  if (!b->desc || !b->indptr || !b->indices || !b->data || !b->c || !b->c0 || !b->q || !b->l || !b->u)
    return fail(h, DVH_ERR_ARG, "null device array in packed batch");
  DVH_HIP(h, hipSetDevice(h->device));
  hipStream_t s = h->stream;
  // the windows' descriptors must describe exactly this LP shape, inside the arrays (the kernel writes through them)
  std::vector<int64_t> desc(8 * (size_t)g->G);
  DVH_HIP(h, hipMemcpyAsync(desc.data(), b->desc + 8 * (int64_t)first, desc.size() * sizeof(int64_t),
                            hipMemcpyDeviceToHost, s));
  // the demand-charge rows' steps and tau columns index the window's base series and columns: range-checked here
  // (an entry >= T or >= J made the kernel read base[] out of bounds and write column indices outside the
  // window), in the same sync as the descriptors
  std::vector<int32_t> dt_((size_t)g->mI), dj_((size_t)g->mI);
  if (g->mI > 0) {
    DVH_HIP(h, hipMemcpyAsync(dt_.data(), g->dcm_t, sizeof(int32_t) * dt_.size(), hipMemcpyDefault, s));
    DVH_HIP(h, hipMemcpyAsync(dj_.data(), g->dcm_j, sizeof(int32_t) * dj_.size(), hipMemcpyDefault, s));
  }
  DVH_HIP(h, hipStreamSynchronize(s));
  for (int32_t i = 0; i < g->mI; ++i)
    if (dt_[i] < 0 || dt_[i] >= g->T || dj_[i] < 0 || dj_[i] >= g->J)
      return fail(h, DVH_ERR_ARG, "battery group: demand-charge row " + std::to_string(i) + " (step " +
                                      std::to_string(dt_[i]) + ", column " + std::to_string(dj_[i]) +
                                      ") outside T = " + std::to_string(g->T) + ", J = " + std::to_string(g->J));
  const bool ice = g->has_ice != 0;
  const int64_t T = g->T, n = (ice ? 5 : 3) * T + g->J, m = T + 1 + g->mI + (ice ? 2 * T : 0),
                nnz = 4 * T + (ice ? 4 : 3) * (int64_t)g->mI + (ice ? 4 * T : 0);
  for (int w = 0; w < g->G; ++w) {
    const int64_t* d = &desc[8 * (size_t)w];
    if (d[0] != n || d[1] != m || d[2] != T + 1 || d[3] != nnz || d[4] < 0 || d[5] < 0 || d[6] < 0 || d[7] < 0 ||
        d[4] + m + 1 > b->total_rows || d[5] + nnz > b->total_nnz || d[6] + n > b->total_n || d[7] + m > b->total_m)
      return fail(h, DVH_ERR_ARG, "battery group: descriptor of window " + std::to_string(first + w) +
                                      " does not match the group's LP shape or the arrays");
  }
  hipError_t e = dvh::launch_build_battery(*g, *b, first, s);
  if (e != hipSuccess) return hip_fail(h, e, "launch_build_battery");
  return DVH_OK;
}

// Medium tier over the candidates of one chunk: plan (structure, segmentation, crossed bounds) -> setup of the
// planned windows (the one-workgroup setup kernel, or grid-wide for n >= kMedSetupNMax) -> team launches: windows of
// up to kChainMedMax segments together, longer ones (the 5-minute annual window) in launches of their own.
// med_done[k] = 1 for the windows solved or reported infeasible; the others stay with the grid-wide path, and so do
// the windows a launch had not finished when it aborted (a segment exchange outlasted the spin limit).
static int chain_pass(dvh_handle* h, const dvh::Batch& b, const dvh::Work& w, const dvh::Chunk& ch,
                      const dvh::Opts& o, const std::vector<int32_t>& med, int max_T,
                      const std::vector<int64_t>& desc, std::vector<char>& med_done, hipStream_t s) {
  const int nm = (int)med.size();
  if (nm == 0) return DVH_OK;
  const size_t I = sizeof(int32_t);
  DVH_HIP(h, h->m_list.ensure(I * (size_t)nm));
  DVH_HIP(h, hipMemcpyAsync(h->m_list.p, med.data(), I * nm, hipMemcpyHostToDevice, s));
  DVH_HIP(h, h->m_plan.ensure(I * (size_t)nm * dvh::kPlanInts));
  hipError_t e = dvh::launch_chain_plan(b, w, ch, h->m_list.as<int32_t>(), nm, max_T, h->m_plan.as<int32_t>(), s);
  if (e != hipSuccess) return hip_fail(h, e, "launch_chain_plan");
  std::vector<int32_t> head((size_t)nm * 4);  // {P, T, J, k} of every plan record
  DVH_HIP(h, hipMemcpy2DAsync(head.data(), 4 * I, h->m_plan.p, I * dvh::kPlanInts, 4 * I, nm, hipMemcpyDeviceToHost, s));
  DVH_HIP(h, sync_stream(h, s));
  std::vector<int32_t> small_setup, accepted;
  for (int i = 0; i < nm; ++i) {
    const int P = head[4 * (size_t)i];
    if (P < 0) med_done[med[i]] = 1;  // crossed bounds: PRIMAL_INFEASIBLE from the plan kernel
    if (P <= 0) continue;
    accepted.push_back(i);
    if (desc[8 * (size_t)med[i]] < dvh::kMedSetupNMax) small_setup.push_back(med[i]);
  }
  if (accepted.empty()) return DVH_OK;
  // setup of the planned windows
  if (!small_setup.empty()) {
    int mn = 0;
    for (int k : small_setup) mn = std::max<int>(mn, (int)desc[8 * (size_t)k]);
    DVH_HIP(h, h->m_pos.ensure(I * small_setup.size()));
    DVH_HIP(h, hipMemcpyAsync(h->m_pos.p, small_setup.data(), I * small_setup.size(), hipMemcpyHostToDevice, s));
    e = dvh::launch_setup_medium(b, w, ch, o, mn, h->m_pos.as<int32_t>(), (int)small_setup.size(), s);
    if (e != hipSuccess) return hip_fail(h, e, "launch_setup_medium");
  }
  for (int i : accepted) {
    const int k = med[i];
    if (desc[8 * (size_t)k] < dvh::kMedSetupNMax) continue;
    e = dvh::launch_setup_long(b, w, ch, o, k, &desc[8 * (size_t)k], s);
    if (e != hipSuccess) return hip_fail(h, e, "launch_setup_long");
  }
  // the one-workgroup setup flags windows it cannot scale (more long rows than its lists): those go grid-wide
  std::vector<double> flag6(accepted.size(), 0.0);
  for (size_t a = 0; a < accepted.size(); ++a)
    DVH_HIP(h, hipMemcpyAsync(&flag6[a], w.scal + (int64_t)(med[accepted[a]] - ch.first) * dvh::kScal + 6,
                              sizeof(double), hipMemcpyDeviceToHost, s));
  DVH_HIP(h, sync_stream(h, s));
  std::vector<int32_t> groups[2];  // plan positions: [0] up to kChainMedMax segments, [1] longer
  int PTg[2] = {0, 0};
  for (size_t a = 0; a < accepted.size(); ++a) {
    if (flag6[a] != 0.0) continue;
    const int i = accepted[a], P = head[4 * (size_t)i];
    const int g = P > dvh::kChainMedMax ? 1 : 0;
    groups[g].push_back(i);
    PTg[g] = std::max(PTg[g], P);
  }
  if (h->chain_cap < 0) {
    int cap = 0;
    if (dvh::chain_capacity(h->device, &cap) != hipSuccess) cap = 0;
    (void)hipGetLastError();
    h->chain_cap = cap;
  }
  if (h->spin_ticks <= 0) {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device) != hipSuccess || khz <= 0) khz = 100000;
    h->spin_ticks = (long long)khz * 1000 * 2;  // 2 s: a partner's hand-off normally takes microseconds
    // DVH_CHAIN_SPIN_TICKS (tests): another limit; < 0 aborts at the first exchange that has to wait, forcing the
    // abort -> grid-wide hand-over path
    if (const char* v = getenv("DVH_CHAIN_SPIN_TICKS")) {
      const long long t = atoll(v);
      if (t != 0) h->spin_ticks = t;
    }
  }
  const int S = h->chain_cap / 8;  // resident slots per XCD
  for (int g = 0; g < 2; ++g) {
    const int PT = PTg[g];
    if (groups[g].empty()) continue;
    const int NT = S >= 1 && PT <= 8 * S ? dvh::chain_team_count(S, PT) : 0;
    if (NT < 1) continue;  // cannot keep a team resident: the grid-wide path takes them
    constexpr int kMaxPerLaunch = 0x3FFF - 2;  // window tags keep 14 bits of a team's window count
    for (size_t a0 = 0; a0 < groups[g].size(); a0 += kMaxPerLaunch) {
      const int np = (int)std::min<size_t>(kMaxPerLaunch, groups[g].size() - a0);
      const int32_t* pos = groups[g].data() + a0;
      std::vector<int32_t> ks(np);
      for (int q = 0; q < np; ++q) ks[q] = med[pos[q]];
      DVH_HIP(h, h->m_pos.ensure(I * 2 * (size_t)np));
      int32_t* dpos = h->m_pos.as<int32_t>();
      DVH_HIP(h, hipMemcpyAsync(dpos, pos, I * np, hipMemcpyHostToDevice, s));
      DVH_HIP(h, hipMemcpyAsync(dpos + np, ks.data(), I * np, hipMemcpyHostToDevice, s));
      e = dvh::launch_chain_mark(b, dpos + np, np, s);
      if (e != hipSuccess) return hip_fail(h, e, "launch_chain_mark");
      DVH_HIP(h, h->m_xbuf.ensure(dvh::chain_xbuf_bytes(NT, PT)));
      DVH_HIP(h, h->m_abort.ensure(dvh::chain_abort_bytes(S)));
      e = dvh::launch_chain(b, w, ch, o, dpos, np, h->m_plan.as<int32_t>(), PT, S, h->m_xbuf.p,
                            h->m_abort.as<int32_t>(), h->spin_ticks, s);
      if (e == hipErrorCooperativeLaunchTooLarge) {  // not resident after all: leave them to the grid-wide path
        (void)hipGetLastError();
        h->chain_cap = 0;
        return DVH_OK;
      }
      if (e != hipSuccess) return hip_fail(h, e, "launch_chain");
      std::vector<int32_t> ab(dvh::chain_abort_bytes(S) / I);
      DVH_HIP(h, hipMemcpyAsync(ab.data(), h->m_abort.p, I * ab.size(), hipMemcpyDeviceToHost, s));
      DVH_HIP(h, sync_stream(h, s));
      if (getenv("DVH_CHAIN_PROBE_DUMP")) {  // timing probe builds: wave 0's waits per workgroup (wall-clock ticks)
        for (int gb = 0; gb < 8 * S; ++gb)
          if (ab[16 + 8 * (size_t)gb + 6] || ab[16 + 8 * (size_t)gb + 7])
            fprintf(stderr, "PROBE block %d tauwait %d hopwait %d\n", gb, ab[16 + 8 * (size_t)gb + 6],
                    ab[16 + 8 * (size_t)gb + 7]);
      }
      if (ab[0] != 0) {
        // a segment exchange outlasted the spin limit: the windows the launch finished keep their results, the
        // others (still marked pending) go to the grid-wide path; the diagnostics stay readable in dvh_last_error
        std::string msg = "medium tier: a segment exchange timed out (PT " + std::to_string(PT) + ", NT " +
                          std::to_string(NT) + "); unfinished windows moved to the grid-wide path; workgroups "
                          "{block: state list round entry tag seen}:";
        for (int gb = 0; gb < 8 * S; ++gb) {
          const int32_t* d = &ab[16 + 8 * (size_t)gb];
          if (d[0] == 0) continue;
          char buf[128];
          snprintf(buf, sizeof buf, " %d: %d %d %d 0x%x 0x%x 0x%x;", gb, d[0], d[1], d[2], d[3], d[4], d[5]);
          msg += buf;
        }
        h->warn += msg;
        ++h->n_chain_aborts;
        std::vector<int32_t> st(2);
        for (int q = 0; q < np; ++q) {
          DVH_HIP(h, hipMemcpy(st.data(), b.istats + 2 * (int64_t)ks[q], 2 * I, hipMemcpyDeviceToHost));
          if (st[0] != dvh::kChainPending) {
            med_done[ks[q]] = 1;
            ++h->n_chain;
          }
        }
        continue;
      }
      for (int q = 0; q < np; ++q) med_done[ks[q]] = 1;
      h->n_chain += np;
    }
  }
  return DVH_OK;
}

// Solve a packed device batch given a host copy of its descriptors.
// The default kernel cascade over one chunk's small windows, its lists formed on the device (dvh_route.hip): the
// battery-banded kernel over the chunk -> its refusals (status -2) through the band-ICE form (both scale the windows
// they take themselves: no setup_kernel for them) -> what that refuses, set up (setup_kernel over the list), through
// the ELL kernels, in two size classes (the small market-day kernels' shapes, n <= 512 and m <= 768, and the
// rest), each instantiation sized for its class -> what they refuse (-1) or cannot hold through the generic CSR
// kernel, both classes in one launch.
// One small read-back per stage that ran ({count, ELL widths, max n / m / nnz} of the windows it hands on; two after
// the ICE form when it refuses windows: their count, then their size classes once they are set up); a batch the band
// kernel takes whole waits once.
static int device_cascade(dvh_handle* h, const dvh::Batch& b, const dvh::Work& w, const dvh::Chunk& ch,
                          const dvh::Opts& o, int nsmall, int wc, int mn, int mm, hipStream_t s,
                          const int32_t* order = nullptr) {
  const size_t I = sizeof(int32_t);
  int32_t* L[5];
  for (int r = 0; r < 5; ++r) L[r] = h->d_list.as<int32_t>() + (size_t)r * wc;
  int32_t* info = h->d_route.as<int32_t>();  // 8 ints per route: {count, wx, wy, max n, max m, max nnz}
  int32_t* rh = h->route_host;
  if (h->cus <= 0 && hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess)
    h->cus = 256;
  // band kernel form: three steps per lane (two windows per CU) once the windows outnumber the CUs; a window alone
  // on its CU is faster in the one-step form (0.75 vs 0.97 us per iteration, profiles/r02x_band_forms.log)
  const int forced_form = h->kernel_path == 3 ? 1 : h->kernel_path == 4 ? 3 : 0;
  auto form_for = [&](int nl) { return forced_form ? forced_form : (nl <= h->cus ? 1 : 3); };
  // route: the windows of `in` (or the chunk) with status `want` and size class `cls` -> L[out], info slot `slot`
  auto route = [&](int slot, const int32_t* in, int n_in, int want, int cls, int out) -> hipError_t {
    return dvh::launch_route(b.desc, b.istats, w.scal, ch.first, n_in, in, want, dvh::kSmallMax, cls, 512, 768,
                             L[out], info + 8 * slot, s);
  };
  auto readback = [&](int slot0, int nslots) -> hipError_t {
    hipError_t e = hipMemcpyAsync(rh + 8 * slot0, info + 8 * slot0, 8 * I * nslots, hipMemcpyDeviceToHost, s);
    return e != hipSuccess ? e : sync_stream(h, s);
  };
  int variant = -1, bvar = -1;
  // the battery forms iterate on [0, 1]-normalised boxes (dvh_band.hip BOX; bench 246.4k vs 239.7k windows/s,
  // profiles/r04m_ab_band_box.log); the few windows with an unbounded ch / dis / ene column (status -3) are re-run by
  // the plain form, which takes every one of them (same structure and scaling checks), after the same read-back.
  // The ICE form's box (elec / on too) is opt-in: it spills as much as the plain ICE form and ran 0.8 % slower on
  // config 5 (profiles/r04n_ab_ice_box.log).  DVH_BAND_BOX: 0 none, 1 (default) battery forms, 2 battery + ICE.
  const char* box_env = getenv("DVH_BAND_BOX");
  const int box_mode = box_env ? atoi(box_env) : 1;
  const bool box = box_mode >= 1, box_ice = box_mode >= 2;
  // (order: the chunk's windows in the caller's launch order, dvh_set_launch_order; the results do not depend on it)
  DVH_HIP(h, dvh::launch_pdhg_band(b, w, ch, o, s, false, form_for(ch.count), box, order, order ? ch.count : 0, &bvar));
  DVH_HIP(h, route(0, nullptr, ch.count, -2, 0, 0));
  if (box) DVH_HIP(h, route(1, nullptr, ch.count, -3, 0, 1));
  DVH_HIP(h, readback(0, box ? 2 : 1));
  if (box && rh[8] > 0) {
    // the plain form over the windows without a box; it can refuse some of them itself (-2: factors outside float's
    // range, checked after scaling, which the box form never reached for them), so the -2 list is formed again, over
    // the chunk, once it has run -- one more read-back, only when such windows exist
    DVH_HIP(h, dvh::launch_pdhg_band(b, w, ch, o, s, false, form_for(rh[8]), false, L[1], rh[8], nullptr));
    DVH_HIP(h, route(0, nullptr, ch.count, -2, 0, 0));
    DVH_HIP(h, readback(0, 1));
  }
  int cur = rh[0];
  h->n_band += nsmall - cur;
  if (nsmall - cur > 0) variant = bvar;
  if (cur > 0) {  // pass 2: the band kernel's ICE form over pass 1's refusals
    DVH_HIP(h, dvh::launch_pdhg_band(b, w, ch, o, s, true, form_for(cur), box_ice, L[0], cur, &bvar));
    DVH_HIP(h, route(1, L[0], cur, -2, 0, 4));
    if (box_ice) DVH_HIP(h, route(2, L[0], cur, -3, 0, 1));
    DVH_HIP(h, readback(1, box_ice ? 2 : 1));
    if (box_ice && rh[16] > 0) {  // the plain ICE form over the ICE windows without a box; its -2s listed again
      DVH_HIP(h, dvh::launch_pdhg_band(b, w, ch, o, s, true, form_for(rh[16]), false, L[1], rh[16], nullptr));
      DVH_HIP(h, route(1, L[0], cur, -2, 0, 4));
      DVH_HIP(h, readback(1, 1));
    }
    const int left = rh[8];
    h->n_band += cur - left;
    if (cur - left > 0 && variant < 0) variant = bvar;
    cur = left;
    if (cur > 0) {
      // what the band kernels refused, set up (the ELL / generic kernels and the ELL widths of the route statistics
      // read setup_kernel's outputs) and handed on by size class
      DVH_HIP(h, dvh::launch_setup(b, w, ch, o, mn, mm, s, L[4], cur));
      DVH_HIP(h, route(1, L[4], cur, -2, 1, 2));
      DVH_HIP(h, route(2, L[4], cur, -2, 2, 3));
      DVH_HIP(h, readback(1, 2));
    }
  }
  if (cur == 0) {
    h->last_variant = variant;
    return DVH_OK;
  }
  // ELL per size class (class c's windows in L[2 + c], info slot 1 + c; refusals -> L[c], the consumed lists)
  int ran[2] = {0, 0};
  for (int c = 0; c < 2; ++c) {
    const int32_t* in = rh + 8 * (1 + c);
    if (in[0] == 0) continue;
    int ev = -1;
    hipError_t e = dvh::launch_pdhg_ell(b, w, ch, o, in[3], in[4], in[1], in[2], s, &ev, L[2 + c], in[0],
                                        in[0] <= 2 * h->cus);
    if (e == hipSuccess) {
      if (variant < 0) variant = ev;
      DVH_HIP(h, route(3 + c, L[2 + c], in[0], -1, 0, c));
      ran[c] = 1;
    } else if (e == hipErrorInvalidValue) {  // no ELL instantiation holds this class: all generic
      (void)hipGetLastError();
    } else {
      return hip_fail(h, e, "launch_pdhg_ell");
    }
  }
  if (ran[0] || ran[1]) DVH_HIP(h, readback(3, 2));
  // the generic kernel over what is left of both classes, in one launch (one window per CU; a window's time does not
  // depend on the other windows', so the classes overlap inside the launch), sized for the windows it gets
  int gn = 0, gm[3] = {0, 0, 0};
  int32_t* gl = nullptr;
  for (int c = 0; c < 2; ++c) {
    const int32_t* in = rh + 8 * (1 + c);
    if (in[0] == 0) continue;
    const int32_t* g = ran[c] ? rh + 8 * (3 + c) : in;  // this class's windows for the generic kernel, their sizes
    int32_t* l = ran[c] ? L[c] : L[2 + c];
    if (ran[c]) h->n_ell += in[0] - g[0];
    if (g[0] == 0) continue;
    if (!gl) {
      gl = l;
    } else {  // append to the first class's list (disjoint subsets of the chunk: fits its wc slots)
      DVH_HIP(h, hipMemcpyAsync(gl + gn, l, I * g[0], hipMemcpyDeviceToDevice, s));
    }
    gn += g[0];
    for (int u = 0; u < 3; ++u) gm[u] = std::max(gm[u], (int)g[3 + u]);
  }
  if (gn > 0) {
    DVH_HIP(h, dvh::launch_power(b, w, ch, o, gl, gn, s));
    int gv = -1;
    hipError_t e = dvh::launch_pdhg(b, w, ch, o, gm[0], gm[1], gm[2], s, &gv, gl, gn);
    if (e == hipErrorInvalidValue)
      return fail(h, DVH_ERR_UNSUPPORTED, "window too large for the on-chip PDHG kernels (n or m > 4096)");
    if (e != hipSuccess) return hip_fail(h, e, "launch_pdhg");
    h->n_generic += gn;
    if (variant < 0) variant = gv;
  }
  h->last_variant = variant;
  return DVH_OK;
}

static int solve_packed(dvh_handle* h, const dvh_packed* bt, const std::vector<int64_t>& desc, hipStream_t s) {
  const int count = bt->count;
  dvh::Opts o;
  o.eps = h->opts.eps;
  o.eps_obj = h->opts.eps_obj;
  o.step_safety = h->opts.step_safety;
  o.rho = h->opts.reflection;
  o.b_suff = h->opts.restart_sufficient;
  o.b_nec = h->opts.restart_necessary;
  o.b_art = h->opts.restart_artificial;
  o.theta = h->opts.primal_weight_theta;
  o.max_iters = h->opts.max_iters;
  o.check_every = h->opts.check_every;
  o.kkt_every = h->opts.kkt_every;
  o.ruiz_iters = h->opts.ruiz_iters;
  o.power_iters = h->opts.power_iters;
  o.warm = h->opts.warm_start != 0;
  o.kkt_predict = h->opts.kkt_predict;
  o.small_max = dvh::kSmallMax;
  dvh::Batch b{bt->desc, bt->indptr, bt->indices, bt->data, bt->c, bt->c0, bt->q, bt->l, bt->u,
               bt->x, bt->y, bt->stats, bt->istats};
  // chunking + workspace sizing
  struct C {
    dvh::Chunk ch;
    int64_t sn, sm, snz;
    int mn, mm;      // maxima over the chunk's small windows (the on-chip kernels' LDS sizing)
    int64_t mnz;
    int nsmall;
    std::vector<int32_t> med;  // medium-tier candidates of the chunk
    int med_n = 0, med_T = 0;
  };
  auto is_large = [&](int k) {
    const int64_t* d = &desc[8 * (size_t)k];
    return d[0] > dvh::kSmallMax || d[1] > dvh::kSmallMax;
  };
  // medium tier candidates: battery-shaped sizes (n = 3T + J, m <= 2T + 1) up to kPMax segments of kChainB steps;
  // the plan kernel verifies the pattern, anything else goes to the grid-wide path
  const bool chain_on = (h->kernel_path == 0 || h->kernel_path >= 3) && o.rho == 1.0 && o.max_iters + o.power_iters < (1 << 17);
  auto is_medium = [&](int k) {
    const int64_t* d = &desc[8 * (size_t)k];
    const int64_t T = d[2] - 1;
    return chain_on && is_large(k) && T > dvh::kChainB && T <= (int64_t)dvh::kPMax * dvh::kChainB &&
           d[0] >= 3 * T && d[0] <= 3 * T + dvh::kChainJMax && d[1] <= 2 * T + 1;
  };
  std::vector<int> large;
  std::vector<char> med_done(count, 0);  // solved (or reported infeasible) by the medium tier
  std::vector<C> chunks;
  int64_t wn = 0, wm = 0, wnz = 0;
  int wc = 0;
  for (int first = 0; first < count; first += kChunkWindows) {
    C c{};
    c.ch.first = first;
    c.ch.count = std::min(kChunkWindows, count - first);
    const int64_t* d0 = &desc[8 * (size_t)first];
    c.ch.base_n = d0[6];
    c.ch.base_m = d0[7];
    c.ch.base_nz = d0[5];
    for (int k = first; k < first + c.ch.count; ++k) {
      const int64_t* d = &desc[8 * (size_t)k];
      c.sn = std::max(c.sn, d[6] + d[0] - c.ch.base_n);
      c.sm = std::max(c.sm, d[7] + d[1] - c.ch.base_m);
      c.snz = std::max(c.snz, d[5] + d[3] - c.ch.base_nz);
      if (is_large(k)) {
        large.push_back(k);
        if (is_medium(k)) {
          c.med.push_back(k);
          c.med_n = std::max<int>(c.med_n, (int)d[0]);
          c.med_T = std::max<int>(c.med_T, (int)d[2] - 1);
        }
        continue;
      }
      ++c.nsmall;
      c.mn = std::max<int>(c.mn, (int)d[0]);
      c.mm = std::max<int>(c.mm, (int)d[1]);
      c.mnz = std::max(c.mnz, d[3]);
    }
    wn = std::max(wn, c.sn);
    wm = std::max(wm, c.sm);
    wnz = std::max(wnz, c.snz);
    wc = std::max(wc, c.ch.count);
    chunks.push_back(c);
  }
  const size_t D = sizeof(double), I = sizeof(int32_t);
  DVH_HIP(h, h->w_tptr.ensure(I * (wn + wc)));
  DVH_HIP(h, h->w_tind.ensure(I * wnz));
  DVH_HIP(h, h->w_tval.ensure(D * wnz));
  DVH_HIP(h, h->w_kval.ensure(D * wnz));
  DVH_HIP(h, h->w_rowof.ensure(I * wnz));
  DVH_HIP(h, h->w_perm.ensure(I * wnz));
  DVH_HIP(h, h->w_dr.ensure(D * wm));
  DVH_HIP(h, h->w_dc.ensure(D * wn));
  DVH_HIP(h, h->w_cs.ensure(D * wn));
  DVH_HIP(h, h->w_ls.ensure(D * wn));
  DVH_HIP(h, h->w_us.ensure(D * wn));
  DVH_HIP(h, h->w_qs.ensure(D * wm));
  DVH_HIP(h, h->w_vbuf.ensure(D * wn));
  DVH_HIP(h, h->w_wbuf.ensure(D * wm));
  DVH_HIP(h, h->w_tmpc.ensure(D * wn));
  DVH_HIP(h, h->w_tmpr.ensure(D * wm));
  DVH_HIP(h, h->w_longk.ensure(I * (size_t)wc * dvh::kLMax));
  DVH_HIP(h, h->w_longt.ensure(I * (size_t)wc * dvh::kLMax));
  DVH_HIP(h, h->w_scal.ensure(D * (size_t)wc * dvh::kScal));
  DVH_HIP(h, h->w_fc.ensure(sizeof(float) * wn));
  DVH_HIP(h, h->w_fr.ensure(sizeof(float) * wm));
  DVH_HIP(h, h->w_queue.ensure(sizeof(int32_t)));
  dvh::Work w{h->w_tptr.as<int32_t>(), h->w_tind.as<int32_t>(), h->w_tval.as<double>(), h->w_kval.as<double>(),
              h->w_rowof.as<int32_t>(), h->w_perm.as<int32_t>(), h->w_dr.as<double>(), h->w_dc.as<double>(),
              h->w_cs.as<double>(), h->w_ls.as<double>(), h->w_us.as<double>(), h->w_qs.as<double>(),
              h->w_vbuf.as<double>(), h->w_wbuf.as<double>(), h->w_tmpc.as<double>(), h->w_tmpr.as<double>(),
              h->w_longk.as<int32_t>(), h->w_longt.as<int32_t>(), h->d_hinv.as<double>(), h->w_scal.as<double>(),
              h->w_fc.as<float>(), h->w_fr.as<float>(), h->w_queue.as<int32_t>(), h->band_slots};
  DVH_HIP(h, h->d_list.ensure(I * 5 * (size_t)wc));  // the cascade's five device lists (dvh_route.hip)
  DVH_HIP(h, h->d_route.ensure(I * 8 * 5));
  if (!h->route_host) DVH_HIP(h, hipHostMalloc((void**)&h->route_host, I * 8 * 5, hipHostMallocDefault));
  h->n_ell = h->n_generic = h->n_large = h->n_band = h->n_chain = 0;
  h->n_chain_aborts = 0;
  h->warn.clear();
  h->large_ms[0] = h->large_ms[1] = 0.0f;
  h->chunk_used = 0;
  DVH_HIP(h, hipEventRecord(h->ev[0], s));
  std::vector<double> scal;
  std::vector<int32_t> ist;
  // dvh_set_launch_order: consumed by this solve; applied when it covers the batch, which is one chunk of small windows
  const int32_t* order = nullptr;
  h->order_used.swap(h->order);
  h->order.clear();
  if (!h->order_used.empty() && (int)h->order_used.size() == count && chunks.size() == 1 && chunks[0].nsmall == count) {
    DVH_HIP(h, h->d_order.ensure(I * count));
    DVH_HIP(h, hipMemcpyAsync(h->d_order.as<int32_t>(), h->order_used.data(), I * count, hipMemcpyHostToDevice, s));
    order = h->d_order.as<int32_t>();
  }
  for (const C& c : chunks) {
    if (c.nsmall == 0 && c.med.empty()) continue;
    if (h->chunk_used == h->chunk_events.size()) {
      std::array<hipEvent_t, 3> ce{nullptr, nullptr, nullptr};
      for (hipEvent_t& e : ce) {
        const hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) {
          for (hipEvent_t x : ce)
            if (x) hipEventDestroy(x);
          return hip_fail(h, r, "hipEventCreate");
        }
      }
      h->chunk_events.push_back(ce);
    }
    const hipEvent_t e0 = h->chunk_events[h->chunk_used][0], e1 = h->chunk_events[h->chunk_used][1],
                     e2 = h->chunk_events[h->chunk_used][2];
    ++h->chunk_used;
    const bool fast = h->kernel_path != 1 && o.rho == 1.0;
    const bool cascade = fast && (h->kernel_path == 0 || h->kernel_path >= 3);
    DVH_HIP(h, hipEventRecord(e0, s));
    // (the device cascade sets up only what the band kernel refuses, inside device_cascade)
    if (c.nsmall > 0 && !cascade) DVH_HIP(h, dvh::launch_setup(b, w, c.ch, o, c.mn, c.mm, s));
    DVH_HIP(h, hipEventRecord(e1, s));
    if (c.nsmall == 0) {
      if (int rc = chain_pass(h, b, w, c.ch, o, c.med, c.med_T, desc, med_done, s)) return rc;
      DVH_HIP(h, hipEventRecord(e2, s));
      continue;
    }
    if (cascade) {
      if (int rc = device_cascade(h, b, w, c.ch, o, c.nsmall, wc, c.mn, c.mm, s, order)) return rc;
      if (int rc = chain_pass(h, b, w, c.ch, o, c.med, c.med_T, desc, med_done, s)) return rc;
      DVH_HIP(h, hipEventRecord(e2, s));
      continue;
    }
    // ---- A/B paths (generic only, ELL -> generic): lists formed on the host
    // ELL widths from the setup statistics (one small D2H per chunk)
    scal.resize((size_t)c.ch.count * dvh::kScal);
    DVH_HIP(h, hipMemcpyAsync(scal.data(), w.scal, sizeof(double) * scal.size(), hipMemcpyDeviceToHost, s));
    DVH_HIP(h, sync_stream(h, s));
    int wx = 0, wy = 0;
    for (int k = 0; k < c.ch.count; ++k) {
      const double* sc = &scal[(size_t)k * dvh::kScal];
      if (sc[6] != 0.0) continue;
      wy = std::max(wy, (int)sc[8]);
      wx = std::max(wx, (int)sc[9]);
    }
    int variant = -1;
    // ELL kernel over the chunk -> generic CSR kernel over the windows it returned (status -1), or the generic kernel
    // alone (kernel path 1, or reflection rho != 1: the fast kernels are specialised to rho = 1).  The band kernels
    // run in the device cascade only.
    hipError_t e = hipErrorInvalidValue;
    if (fast) {
      int ev = -1;
      e = dvh::launch_pdhg_ell(b, w, c.ch, o, c.mn, c.mm, wx, wy, s, &ev, nullptr, 0);
      if (e == hipSuccess) variant = ev;
    }
    std::vector<int32_t> generic;
    if (e == hipSuccess) {
      ist.resize(2 * (size_t)c.ch.count);
      DVH_HIP(h, hipMemcpyAsync(ist.data(), bt->istats + 2 * (size_t)c.ch.first, I * ist.size(),
                                hipMemcpyDeviceToHost, s));
      DVH_HIP(h, sync_stream(h, s));
      int nl = 0;
      for (int k = 0; k < c.ch.count; ++k) {
        if (is_large(c.ch.first + k)) {
          ++nl;
          continue;
        }
        if (ist[2 * (size_t)k] == -1) generic.push_back(c.ch.first + k);
      }
      h->n_ell += c.ch.count - (int)generic.size() - nl;
    } else if (e == hipErrorInvalidValue) {  // the generic path, or no ELL instantiation covers the chunk's sizes
      (void)hipGetLastError();
      for (int k = 0; k < c.ch.count; ++k)
        if (!is_large(c.ch.first + k)) generic.push_back(c.ch.first + k);
    } else {
      return hip_fail(h, e, "launch_pdhg_ell");
    }
    if (!generic.empty()) {
      DVH_HIP(h, hipMemcpyAsync(h->d_list.p, generic.data(), I * generic.size(), hipMemcpyHostToDevice, s));
      DVH_HIP(h, dvh::launch_power(b, w, c.ch, o, h->d_list.as<int32_t>(), (int)generic.size(), s));
      int gv = -1;
      e = dvh::launch_pdhg(b, w, c.ch, o, c.mn, c.mm, c.mnz, s, &gv, h->d_list.as<int32_t>(), (int)generic.size());
      if (e == hipErrorInvalidValue)
        return fail(h, DVH_ERR_UNSUPPORTED, "window too large for the on-chip PDHG kernels (n or m > 4096)");
      if (e != hipSuccess) return hip_fail(h, e, "launch_pdhg");
      h->n_generic += (int)generic.size();
      if (variant < 0) variant = gv;
      DVH_HIP(h, sync_stream(h, s));  // d_list is reused by the next chunk
    }
    if (int rc = chain_pass(h, b, w, c.ch, o, c.med, c.med_T, desc, med_done, s)) return rc;
    DVH_HIP(h, hipEventRecord(e2, s));
    h->last_variant = variant;
  }
  // windows above the on-chip limits that the medium tier did not take: one at a time, the whole GPU each
  for (int k : large) {
    if (med_done[k]) continue;
    if (!h->large) h->large = dvh::large_create();
    std::string msg;
    hipError_t e = dvh::large_solve(h->large, b, k, &desc[8 * (size_t)k], o, h->d_hinv.as<double>(), s, &msg,
                                    &h->large_ms[0], &h->large_ms[1]);
    if (e != hipSuccess) return fail(h, DVH_ERR_HIP, "window " + std::to_string(k) + ": " + msg);
    ++h->n_large;
  }
  DVH_HIP(h, hipEventRecord(h->ev[3], s));
  return DVH_OK;
}

static int finish_timing(dvh_handle* h, hipStream_t s) {
  DVH_HIP(h, sync_stream(h, s));
  float t = 0;
  h->timing[0] = h->timing[1] = h->timing[2] = 0;
  if (hipEventElapsedTime(&t, h->ev[0], h->ev[3]) == hipSuccess) h->timing[0] = t;
  for (size_t i = 0; i < h->chunk_used; ++i) {
    const auto& ce = h->chunk_events[i];
    if (hipEventElapsedTime(&t, ce[0], ce[1]) == hipSuccess) h->timing[1] += t;
    if (hipEventElapsedTime(&t, ce[1], ce[2]) == hipSuccess) h->timing[2] += t;
  }
  h->timing[1] += h->large_ms[0];
  h->timing[2] += h->large_ms[1];
  return DVH_OK;
}

static int solve_batch_one(dvh_handle* h, const dvh_lp* lps, int32_t count, dvh_result* out);

// Contiguous, cost-balanced ranges of the batch for the handle's devices (windows the on-chip kernels take cost one
// workgroup each; larger windows run grid-wide and cost in proportion to their nonzeros; dervet_hip/parallel.py
// window_cost / shard_weighted are the same rule for ranks).
static std::vector<int> split_batch(const dvh_lp* lps, int32_t count, int parts) {
  std::vector<double> cum(count + 1, 0.0);
  for (int k = 0; k < count; ++k) {
    const dvh_lp& lp = lps[k];
    const bool big = lp.n > dvh::kSmallMax || lp.m_eq + lp.m_ineq > dvh::kSmallMax;
    cum[k + 1] = cum[k] + (big ? std::max(1.0, lp.nnz / 5208.0) : 1.0);
  }
  std::vector<int> b(parts + 1, count);
  b[0] = 0;
  for (int r = 1; r < parts; ++r) {
    const double target = cum[count] * r / parts;
    int k = b[r - 1];
    while (k < count && cum[k] + 0.5 * (cum[k + 1] - cum[k]) < target) ++k;
    b[r] = k;
  }
  return b;
}

extern "C" int dvh_solve_batch(dvh_handle* h, const dvh_lp* lps, int32_t count, dvh_result* out) {
  if (!h) return DVH_ERR_ARG;
  if (count < 0 || (count > 0 && (!lps || !out))) return fail(h, DVH_ERR_ARG, "null lps/out or negative count");
  if (count == 0) return DVH_OK;
  if (h->peers.empty()) return solve_batch_one(h, lps, count, out);
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<dvh_handle*> hs = {h};
  hs.insert(hs.end(), h->peers.begin(), h->peers.end());
  const int P = (int)hs.size();
  const std::vector<int> b = split_batch(lps, count, P);
  std::vector<int> rc(P, DVH_OK);
  std::vector<std::thread> th;
  for (int i = 1; i < P; ++i)
    if (b[i + 1] > b[i]) th.emplace_back([&, i] { rc[i] = solve_batch_one(hs[i], lps + b[i], b[i + 1] - b[i], out + b[i]); });
  if (b[1] > b[0]) rc[0] = solve_batch_one(h, lps, b[1], out);
  for (auto& t : th) t.join();
  int nell = 0, ngen = 0, nlarge = 0, nband = 0, nchain = 0, naborts = 0;
  std::string warn;
  double setup = 0.0, pdhg = 0.0;
  for (int i = 0; i < P; ++i) {
    if (rc[i] != DVH_OK) {
      const std::string msg = hs[i]->err;  // copy first: hs[0] is h
      return fail(h, rc[i], "device " + std::to_string(hs[i]->device) + " (part " + std::to_string(i) + "): " + msg);
    }
    if (b[i + 1] == b[i]) continue;
    nell += hs[i]->n_ell;
    ngen += hs[i]->n_generic;
    nlarge += hs[i]->n_large;
    nband += hs[i]->n_band;
    nchain += hs[i]->n_chain;
    naborts += hs[i]->n_chain_aborts;
    warn += hs[i]->warn;
    setup = std::max(setup, hs[i]->timing[1]);
    pdhg = std::max(pdhg, hs[i]->timing[2]);
  }
  h->n_ell = nell;
  h->n_generic = ngen;
  h->n_large = nlarge;
  h->n_band = nband;
  h->n_chain = nchain;
  h->n_chain_aborts = naborts;
  h->warn = warn;
  h->timing[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  h->timing[1] = setup;
  h->timing[2] = pdhg;
  return DVH_OK;
}

static int solve_batch_one(dvh_handle* h, const dvh_lp* lps, int32_t count, dvh_result* out) {
  DVH_HIP(h, hipSetDevice(h->device));
  std::vector<int64_t> desc(8 * (size_t)count);
  int64_t tn = 0, tm = 0, tz = 0, tr = 0;
  for (int k = 0; k < count; ++k) {
    std::string msg = dvh::validate_lp(lps[k], k);
    if (!msg.empty()) return fail(h, DVH_ERR_ARG, msg);
    const dvh_lp& lp = lps[k];
    const int m = lp.m_eq + lp.m_ineq;
    int64_t* d = &desc[8 * (size_t)k];
    d[0] = lp.n;
    d[1] = m;
    d[2] = lp.m_eq;
    d[3] = lp.nnz;
    d[4] = tr;
    d[5] = tz;
    d[6] = tn;
    d[7] = tm;
    tr += m + 1;
    tz += lp.nnz;
    tn += lp.n;
    tm += m;
  }
  std::vector<int32_t> indptr(tr), indices(tz);
  std::vector<double> data(tz), c(tn), l(tn), u(tn), q(tm), c0(count);
  for (int k = 0; k < count; ++k) {
    const dvh_lp& lp = lps[k];
    const int64_t* d = &desc[8 * (size_t)k];
    const int m = (int)d[1];
    std::memcpy(&indptr[d[4]], lp.indptr, sizeof(int32_t) * (m + 1));
    if (lp.nnz) {
      std::memcpy(&indices[d[5]], lp.indices, sizeof(int32_t) * lp.nnz);
      std::memcpy(&data[d[5]], lp.data, sizeof(double) * lp.nnz);
    }
    std::memcpy(&c[d[6]], lp.c, sizeof(double) * lp.n);
    std::memcpy(&l[d[6]], lp.l, sizeof(double) * lp.n);
    std::memcpy(&u[d[6]], lp.u, sizeof(double) * lp.n);
    if (m) std::memcpy(&q[d[7]], lp.q, sizeof(double) * m);
    c0[k] = lp.c0;
  }
  const size_t D = sizeof(double), I = sizeof(int32_t);
  DVH_HIP(h, h->d_desc.ensure(desc.size() * sizeof(int64_t)));
  DVH_HIP(h, h->d_indptr.ensure(I * tr));
  DVH_HIP(h, h->d_indices.ensure(I * std::max<int64_t>(tz, 1)));
  DVH_HIP(h, h->d_data.ensure(D * std::max<int64_t>(tz, 1)));
  DVH_HIP(h, h->d_c.ensure(D * tn));
  DVH_HIP(h, h->d_l.ensure(D * tn));
  DVH_HIP(h, h->d_u.ensure(D * tn));
  DVH_HIP(h, h->d_x.ensure(D * tn));
  DVH_HIP(h, h->d_q.ensure(D * std::max<int64_t>(tm, 1)));
  DVH_HIP(h, h->d_y.ensure(D * std::max<int64_t>(tm, 1)));
  DVH_HIP(h, h->d_c0.ensure(D * count));
  DVH_HIP(h, h->d_stats.ensure(D * 4 * count));
  DVH_HIP(h, h->d_istats.ensure(I * 2 * count));
  hipStream_t s = h->stream;
  DVH_HIP(h, hipMemcpyAsync(h->d_desc.p, desc.data(), desc.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipMemcpyAsync(h->d_indptr.p, indptr.data(), I * tr, hipMemcpyHostToDevice, s));
  if (tz) {
    DVH_HIP(h, hipMemcpyAsync(h->d_indices.p, indices.data(), I * tz, hipMemcpyHostToDevice, s));
    DVH_HIP(h, hipMemcpyAsync(h->d_data.p, data.data(), D * tz, hipMemcpyHostToDevice, s));
  }
  DVH_HIP(h, hipMemcpyAsync(h->d_c.p, c.data(), D * tn, hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipMemcpyAsync(h->d_l.p, l.data(), D * tn, hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipMemcpyAsync(h->d_u.p, u.data(), D * tn, hipMemcpyHostToDevice, s));
  if (tm) DVH_HIP(h, hipMemcpyAsync(h->d_q.p, q.data(), D * tm, hipMemcpyHostToDevice, s));
  DVH_HIP(h, hipMemcpyAsync(h->d_c0.p, c0.data(), D * count, hipMemcpyHostToDevice, s));
  std::vector<double> x0, y0;
  if (h->opts.warm_start) {  // starting points: the caller's x / y buffers (zero where absent)
    x0.assign(tn, 0.0);
    y0.assign(std::max<int64_t>(tm, 1), 0.0);
    for (int k = 0; k < count; ++k) {
      const int64_t* d = &desc[8 * (size_t)k];
      if (out[k].x) std::memcpy(&x0[d[6]], out[k].x, D * d[0]);
      if (out[k].y && d[1]) std::memcpy(&y0[d[7]], out[k].y, D * d[1]);
    }
    DVH_HIP(h, hipMemcpyAsync(h->d_x.p, x0.data(), D * tn, hipMemcpyHostToDevice, s));
    DVH_HIP(h, hipMemcpyAsync(h->d_y.p, y0.data(), D * y0.size(), hipMemcpyHostToDevice, s));
  }
  dvh_packed bt{};
  bt.count = count;
  bt.total_n = tn;
  bt.total_m = tm;
  bt.total_nnz = tz;
  bt.total_rows = tr;
  bt.desc = h->d_desc.as<int64_t>();
  bt.indptr = h->d_indptr.as<int32_t>();
  bt.indices = h->d_indices.as<int32_t>();
  bt.data = h->d_data.as<double>();
  bt.c = h->d_c.as<double>();
  bt.c0 = h->d_c0.as<double>();
  bt.q = h->d_q.as<double>();
  bt.l = h->d_l.as<double>();
  bt.u = h->d_u.as<double>();
  bt.x = h->d_x.as<double>();
  bt.y = h->d_y.as<double>();
  bt.stats = h->d_stats.as<double>();
  bt.istats = h->d_istats.as<int32_t>();
  h->n_syncs = 0;
  int rc = solve_packed(h, &bt, desc, s);
  if (rc != DVH_OK) return rc;
  std::vector<double> x(tn), y(tm), stats(4 * (size_t)count);
  std::vector<int32_t> ist(2 * (size_t)count);
  DVH_HIP(h, hipMemcpyAsync(x.data(), h->d_x.p, D * tn, hipMemcpyDeviceToHost, s));
  if (tm) DVH_HIP(h, hipMemcpyAsync(y.data(), h->d_y.p, D * tm, hipMemcpyDeviceToHost, s));
  DVH_HIP(h, hipMemcpyAsync(stats.data(), h->d_stats.p, D * 4 * count, hipMemcpyDeviceToHost, s));
  DVH_HIP(h, hipMemcpyAsync(ist.data(), h->d_istats.p, I * 2 * count, hipMemcpyDeviceToHost, s));
  rc = finish_timing(h, s);
  if (rc != DVH_OK) return rc;
  for (int k = 0; k < count; ++k) {
    const int64_t* d = &desc[8 * (size_t)k];
    dvh_result& r = out[k];
    if (r.x) std::memcpy(r.x, &x[d[6]], D * d[0]);
    if (r.y && d[1]) std::memcpy(r.y, &y[d[7]], D * d[1]);
    r.obj = stats[4 * k];
    r.primal_res_rel = stats[4 * k + 1];
    r.dual_res_rel = stats[4 * k + 2];
    r.gap_rel = stats[4 * k + 3];
    r.status = ist[2 * k];
    r.iters = ist[2 * k + 1];
  }
  return DVH_OK;
}

extern "C" int dvh_solve_packed_device(dvh_handle* h, const dvh_packed* bt, void* stream) {
  if (!h) return DVH_ERR_ARG;
  if (!bt || bt->count < 0) return fail(h, DVH_ERR_ARG, "null or negative batch");
  if (bt->count == 0) return DVH_OK;
  if (!bt->desc || !bt->indptr || !bt->c || !bt->c0 || !bt->l || !bt->u || !bt->x || !bt->stats || !bt->istats)
    return fail(h, DVH_ERR_ARG, "null device array in packed batch");
  DVH_HIP(h, hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  h->n_syncs = 0;
  std::vector<int64_t> desc(8 * (size_t)bt->count);
  DVH_HIP(h, hipMemcpyAsync(desc.data(), bt->desc, desc.size() * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  DVH_HIP(h, sync_stream(h, s));
  // host-side sanity of the descriptors (no device data is read beyond desc)
  for (int k = 0; k < bt->count; ++k) {
    const int64_t* d = &desc[8 * (size_t)k];
    if (d[0] <= 0 || d[1] < 0 || d[2] < 0 || d[2] > d[1] || d[3] < 0 || d[4] < 0 || d[5] < 0 || d[6] < 0 || d[7] < 0 ||
        d[4] + d[1] + 1 > bt->total_rows || d[5] + d[3] > bt->total_nnz || d[6] + d[0] > bt->total_n ||
        d[7] + d[1] > bt->total_m)
      return fail(h, DVH_ERR_ARG, "packed descriptor " + std::to_string(k) + " out of range");
    if (k > 0) {
      const int64_t* p = &desc[8 * (size_t)(k - 1)];
      if (d[5] < p[5] || d[6] < p[6] || d[7] < p[7])
        return fail(h, DVH_ERR_ARG, "packed descriptors must have non-decreasing offsets");
    }
  }
  int rc = solve_packed(h, bt, desc, s);
  if (rc != DVH_OK) return rc;
  return finish_timing(h, s);
}

// ORACLE / CPU BASELINE (test infrastructure, not the product): the batched PDHG of libdervet_hip restated in plain
// C++ for host cores, behind the same C ABI (include/dervet_hip.h; the core entry points -- create / destroy /
// options / dvh_solve_batch / timing; device-only entry points return DVH_ERR_UNSUPPORTED).
//
// It is the algorithm of oracle/pdlp_ref.py (restarted reflected Halpern PDHG, Ruiz + Pock-Chambolle scaling,
// power-iteration step size, adaptive restarts, primal weight, relative-KKT + objective-error termination) on CSR
// with sequential sums, one window per OpenMP thread.  Uses: the second CPU baseline of bench.py (the same
// iterations on host cores, beside HiGHS), and a GPU-less run of the whole ctypes stack (tests/test_cpu_pdhg.py).
// The product library never loads it: dervet_hip/_lib.py loads libdervet_hip.so only, and fails without it.
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../include/dervet_hip.h"
// the product's host-side input validation (plain C++, der-vet_amd/csrc/dvh_validate.cpp), compiled in by build()
#include "../der-vet_amd/csrc/dvh_validate.h"

struct dvh_handle {
  dvh_options opts;
  std::string err;
  double timing[3] = {0, 0, 0};
  int threads = 0;
};

namespace {

struct Csr {
  int rows = 0, cols = 0;
  std::vector<int> p, j;
  std::vector<double> v;
  void matvec(const double* x, double* y) const {  // y = A x
    for (int r = 0; r < rows; ++r) {
      double s = 0.0;
      for (int k = p[r]; k < p[r + 1]; ++k) s += v[k] * x[j[k]];
      y[r] = s;
    }
  }
};

Csr transpose(const Csr& a) {  // rows of the result in ascending original-row order
  Csr t;
  t.rows = a.cols;
  t.cols = a.rows;
  t.p.assign(a.cols + 1, 0);
  for (int k = 0; k < a.p[a.rows]; ++k) ++t.p[a.j[k] + 1];
  for (int c = 0; c < a.cols; ++c) t.p[c + 1] += t.p[c];
  t.j.resize(a.p[a.rows]);
  t.v.resize(a.p[a.rows]);
  std::vector<int> cur(t.p.begin(), t.p.end() - 1);
  for (int r = 0; r < a.rows; ++r)
    for (int k = a.p[r]; k < a.p[r + 1]; ++k) {
      const int d = cur[a.j[k]]++;
      t.j[d] = r;
      t.v[d] = a.v[k];
    }
  return t;
}

double norm2(const std::vector<double>& a) {
  double s = 0.0;
  for (double x : a) s += x * x;
  return std::sqrt(s);
}

struct Out {
  std::vector<double> x, y;
  double obj = 0, pres = 0, dres = 0, gap = 0;
  int status = DVH_ITER_LIMIT, iters = 0;
};

void solve_one(const dvh_lp& lp, const dvh_options& o, const double* x0, const double* y0, Out& out) {
  const int n = lp.n, m = lp.m_eq + lp.m_ineq, me = lp.m_eq;
  out.x.assign(n, 0.0);
  out.y.assign(m, 0.0);
  for (int j = 0; j < n; ++j)
    if (lp.l[j] > lp.u[j]) {  // crossed bounds: infeasible as given, no iterations (as the GPU setup kernel)
      out.status = DVH_PRIMAL_INFEASIBLE;
      out.obj = NAN;
      return;
    }
  Csr K;
  K.rows = m;
  K.cols = n;
  K.p.assign(lp.indptr, lp.indptr + m + 1);
  K.j.assign(lp.indices, lp.indices + lp.nnz);
  K.v.assign(lp.data, lp.data + lp.nnz);
  // ---- Ruiz (inf-norm) + Pock-Chambolle (alpha = 1) on |K|
  std::vector<double> Dr(m, 1.0), Dc(n, 1.0), rmax(m), cmax(n);
  for (int it = 0; it < o.ruiz_iters; ++it) {
    std::fill(rmax.begin(), rmax.end(), 0.0);
    std::fill(cmax.begin(), cmax.end(), 0.0);
    for (int r = 0; r < m; ++r)
      for (int k = K.p[r]; k < K.p[r + 1]; ++k) {
        const double a = Dr[r] * std::fabs(K.v[k]) * Dc[K.j[k]];
        rmax[r] = std::max(rmax[r], a);
        cmax[K.j[k]] = std::max(cmax[K.j[k]], a);
      }
    for (int r = 0; r < m; ++r) Dr[r] /= std::sqrt(rmax[r] > 0 ? rmax[r] : 1.0);
    for (int c = 0; c < n; ++c) Dc[c] /= std::sqrt(cmax[c] > 0 ? cmax[c] : 1.0);
  }
  std::fill(rmax.begin(), rmax.end(), 0.0);
  std::fill(cmax.begin(), cmax.end(), 0.0);
  for (int r = 0; r < m; ++r)
    for (int k = K.p[r]; k < K.p[r + 1]; ++k) {
      const double a = Dr[r] * std::fabs(K.v[k]) * Dc[K.j[k]];
      rmax[r] += a;
      cmax[K.j[k]] += a;
    }
  for (int r = 0; r < m; ++r) Dr[r] /= std::sqrt(rmax[r] > 0 ? rmax[r] : 1.0);
  for (int c = 0; c < n; ++c) Dc[c] /= std::sqrt(cmax[c] > 0 ? cmax[c] : 1.0);
  Csr Kt = K;
  for (int r = 0; r < m; ++r)
    for (int k = K.p[r]; k < K.p[r + 1]; ++k) Kt.v[k] = Dr[r] * K.v[k] * Dc[K.j[k]];
  const Csr KtT = transpose(Kt);
  std::vector<double> ct(n), lt(n), ut(n), qt(m);
  for (int c = 0; c < n; ++c) {
    ct[c] = Dc[c] * lp.c[c];
    lt[c] = lp.l[c] / Dc[c];
    ut[c] = lp.u[c] / Dc[c];
  }
  for (int r = 0; r < m; ++r) qt[r] = Dr[r] * lp.q[r];
  // ---- ||Kt||_2: v <- Kt'(Kt v) from 1/sqrt(n), sigma^2 = |v_P| / |v_{P-1}|
  std::vector<double> v(n, 1.0 / std::sqrt((double)n)), prev(n), tmpm(m), tmpn(n);
  for (int it = 0; it < o.power_iters; ++it) {
    prev = v;
    Kt.matvec(v.data(), tmpm.data());
    KtT.matvec(tmpm.data(), v.data());
  }
  const double a = norm2(prev), b = norm2(v);
  const double eta = o.step_safety / (a > 0 && b > 0 ? std::sqrt(b / a) : 1.0);
  const double nc = norm2(ct), nq = norm2(qt);
  double w = (nc > 1e-10 && nq > 1e-10) ? nc / nq : 1.0;
  double qn = 0, cn = 0;
  for (int r = 0; r < m; ++r) qn += lp.q[r] * lp.q[r];
  for (int c = 0; c < n; ++c) cn += lp.c[c] * lp.c[c];
  qn = std::sqrt(qn);
  cn = std::sqrt(cn);
  // ---- iterate
  std::vector<double> x(n), y(m, 0.0), xa, ya, xp(n), yp(m), xb(n), kty(n), kx(m);
  for (int c = 0; c < n; ++c) x[c] = std::min(std::max(x0 ? x0[c] / Dc[c] : 0.0, lt[c]), ut[c]);
  if (y0)
    for (int r = 0; r < m; ++r) y[r] = r >= me ? std::max(y0[r] / Dr[r], 0.0) : y0[r] / Dr[r];
  if (x0) {  // the band kernels' warm-start weight: geometric mean of the data's and the start's ||y~|| / ||x~||
    double nx = 0, ny = 0;
    for (double v : x) nx += v * v;
    for (double v : y) ny += v * v;
    if (nx > 1e-20 && ny > 1e-20) w = std::sqrt(std::sqrt(ny / nx) * w);
  }
  xa = x;
  ya = y;
  auto T = [&](const std::vector<double>& xi, const std::vector<double>& yi) {
    const double tau = eta / w, sigma = eta * w;
    KtT.matvec(yi.data(), kty.data());
    for (int c = 0; c < n; ++c) {
      xp[c] = std::min(std::max(xi[c] - tau * (ct[c] - kty[c]), lt[c]), ut[c]);
      xb[c] = 2.0 * xp[c] - xi[c];
    }
    Kt.matvec(xb.data(), kx.data());
    for (int r = 0; r < m; ++r) {
      yp[r] = yi[r] + sigma * (qt[r] - kx[r]);
      if (r >= me) yp[r] = std::max(yp[r], 0.0);
    }
  };
  struct Kkt {
    double pres, dres, gap, pobj, dobj, pabs, ynorm, rdx;
  };
  std::vector<double> xs(n), ys(m), res(m), rc(n);
  auto kkt = [&]() {
    for (int c = 0; c < n; ++c) xs[c] = Dc[c] * xp[c];
    for (int r = 0; r < m; ++r) ys[r] = Dr[r] * yp[r];
    K.matvec(xs.data(), res.data());
    double pr = 0, yn = 0, qy = 0;
    for (int r = 0; r < m; ++r) {
      double d = lp.q[r] - res[r];
      if (r >= me) d = std::max(d, 0.0);
      pr += d * d;
      yn += ys[r] * ys[r];
      qy += lp.q[r] * ys[r];
    }
    std::fill(rc.begin(), rc.end(), 0.0);
    for (int r = 0; r < m; ++r)
      for (int k = K.p[r]; k < K.p[r + 1]; ++k) rc[K.j[k]] += K.v[k] * ys[r];
    double dr = 0, cx = 0, bt = 0, rdx = 0;
    for (int c = 0; c < n; ++c) {
      const double g = lp.c[c] - rc[c];
      const bool fl = std::isfinite(lp.l[c]), fh = std::isfinite(lp.u[c]);
      const double lam = (fl && fh) ? g : (fl ? std::max(g, 0.0) : (fh ? std::min(g, 0.0) : 0.0));
      dr += (g - lam) * (g - lam);
      rdx += std::fabs(g - lam) * std::fabs(xs[c]);
      cx += lp.c[c] * xs[c];
      bt += (fl ? lp.l[c] * std::max(lam, 0.0) : 0.0) + (fh ? lp.u[c] * std::min(lam, 0.0) : 0.0);
    }
    Kkt k;
    k.pobj = cx + lp.c0;
    k.dobj = qy + bt + lp.c0;
    k.pabs = std::sqrt(pr);
    k.ynorm = std::sqrt(yn);
    k.rdx = rdx;
    k.pres = k.pabs / (1.0 + qn);
    k.dres = std::sqrt(dr) / (1.0 + cn);
    k.gap = std::fabs(k.pobj - k.dobj) / (1.0 + std::fabs(k.pobj) + std::fabs(k.dobj));
    return k;
  };
  int it = 0, kin = 0;
  double r0 = -1.0, rprev = -1.0;
  Kkt last{};
  bool have = false;
  std::vector<double> lx = x, ly = y;
  while (it < o.max_iters) {
    T(x, y);
    ++it;
    if (it % o.check_every == 0) {
      double dx2 = 0, dy2 = 0;
      for (int c = 0; c < n; ++c) dx2 += (x[c] - xp[c]) * (x[c] - xp[c]);
      for (int r = 0; r < m; ++r) dy2 += (y[r] - yp[r]) * (y[r] - yp[r]);
      const double r = std::sqrt(w * dx2 + dy2 / w);
      if (it % (o.check_every * o.kkt_every) == 0 || it + o.check_every > o.max_iters) {
        last = kkt();
        have = true;
        lx = xp;
        ly = yp;
        // objective gate (csrc/dvh_device.h kkt_done): gap + ||y|| ||r_p|| + sum_j |r_d,j| |x_j|
        const bool obj_ok = !(o.eps_obj > 0.0) || std::fabs(last.pobj - last.dobj) + last.ynorm * last.pabs + last.rdx <=
                                                       o.eps_obj * (1.0 + std::fabs(last.pobj));
        if (last.pres <= o.eps && last.dres <= o.eps && last.gap <= o.eps && obj_ok) {
          out.status = DVH_OPTIMAL;
          break;
        }
        if (!(std::isfinite(last.pobj) && std::isfinite(last.dobj))) {
          out.status = DVH_NUMERICAL;
          break;
        }
      }
      if (r0 < 0.0) r0 = r;
      const bool restart = (r <= o.restart_sufficient * r0) || (r <= o.restart_necessary * r0 && rprev >= 0.0 && r > rprev) ||
                           (kin + 1 >= o.restart_artificial * it);
      if (restart) {
        double ddx = 0, ddy = 0;
        for (int c = 0; c < n; ++c) ddx += (xp[c] - xa[c]) * (xp[c] - xa[c]);
        for (int rr = 0; rr < m; ++rr) ddy += (yp[rr] - ya[rr]) * (yp[rr] - ya[rr]);
        ddx = std::sqrt(ddx);
        ddy = std::sqrt(ddy);
        if (ddx > 1e-10 && ddy > 1e-10)
          w = std::exp(o.primal_weight_theta * std::log(ddy / ddx) + (1.0 - o.primal_weight_theta) * std::log(w));
        x = xp;
        y = yp;
        xa = xp;
        ya = yp;
        kin = 0;
        r0 = r;
        rprev = -1.0;
        continue;
      }
      rprev = r;
    }
    const double cb = 1.0 / (kin + 2.0), ca = 1.0 - cb, rho = o.reflection;
    for (int c = 0; c < n; ++c) x[c] = ca * ((1.0 + rho) * xp[c] - rho * x[c]) + cb * xa[c];
    for (int r = 0; r < m; ++r) y[r] = ca * ((1.0 + rho) * yp[r] - rho * y[r]) + cb * ya[r];
    ++kin;
  }
  if (out.status != DVH_OPTIMAL || !have) {  // report the last checked point
    if (!have) {
      xp = x;
      yp = y;
      last = kkt();
    } else {
      xp = lx;
      yp = ly;
    }
  }
  out.x.resize(n);
  out.y.resize(m);
  for (int c = 0; c < n; ++c) out.x[c] = Dc[c] * xp[c];
  for (int r = 0; r < m; ++r) out.y[r] = Dr[r] * yp[r];
  double obj = lp.c0;
  for (int c = 0; c < n; ++c) obj += lp.c[c] * out.x[c];
  out.obj = obj;
  out.pres = last.pres;
  out.dres = last.dres;
  out.gap = last.gap;
  out.iters = it;
}

}  // namespace

extern "C" {

const char* dvh_version(void) { return "dervet_hip CPU restatement (oracle/cpu_pdhg.cpp, OpenMP)"; }

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
  o->eps_obj = 1e-6;
}

int dvh_create(int, const dvh_options* opts, dvh_handle** out) {
  if (!out) return DVH_ERR_ARG;
  dvh_handle* h = new dvh_handle();
  dvh_default_options(&h->opts);
  if (opts) h->opts = *opts;
  const char* t = getenv("DVH_CPU_THREADS");
  h->threads = t ? atoi(t) : 0;
  *out = h;
  return DVH_OK;
}

int dvh_create_devices(const int32_t*, int32_t, const dvh_options* opts, dvh_handle** out) {
  return dvh_create(1, opts, out);
}

int dvh_device_count(const dvh_handle* h) { return h ? 1 : 0; }

int dvh_destroy(dvh_handle* h) {
  if (!h) return DVH_ERR_ARG;
  delete h;
  return DVH_OK;
}

const char* dvh_last_error(const dvh_handle* h) { return h ? h->err.c_str() : "null handle"; }

int dvh_set_options(dvh_handle* h, const dvh_options* opts) {
  if (!h || !opts) return DVH_ERR_ARG;
  h->opts = *opts;
  return DVH_OK;
}

int dvh_solve_batch(dvh_handle* h, const dvh_lp* lps, int32_t count, dvh_result* out) {
  if (!h) return DVH_ERR_ARG;
  if (count < 0 || (count > 0 && (!lps || !out))) return DVH_ERR_ARG;
  for (int k = 0; k < count; ++k) {  // the same checks and messages as libdervet_hip's dvh_solve_batch
    std::string msg = dvh::validate_lp(lps[k], k);
    if (!msg.empty()) {
      h->err = msg;
      return DVH_ERR_ARG;
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  const dvh_options o = h->opts;
  if (h->threads > 0) omp_set_num_threads(h->threads);
#pragma omp parallel for schedule(dynamic, 1)
  for (int k = 0; k < count; ++k) {
    Out r;
    solve_one(lps[k], o, o.warm_start ? out[k].x : nullptr, o.warm_start ? out[k].y : nullptr, r);
    if (out[k].x) std::memcpy(out[k].x, r.x.data(), sizeof(double) * r.x.size());
    if (out[k].y && !r.y.empty()) std::memcpy(out[k].y, r.y.data(), sizeof(double) * r.y.size());
    out[k].obj = r.obj;
    out[k].primal_res_rel = r.pres;
    out[k].dual_res_rel = r.dres;
    out[k].gap_rel = r.gap;
    out[k].status = r.status;
    out[k].iters = r.iters;
  }
  h->timing[0] = h->timing[2] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  h->timing[1] = 0.0;
  return DVH_OK;
}

int dvh_last_timing(const dvh_handle* h, double* ms3) {
  if (!h || !ms3) return DVH_ERR_ARG;
  for (int i = 0; i < 3; ++i) ms3[i] = h->timing[i];
  return DVH_OK;
}

// device-only entry points of the header: not part of the CPU restatement
int dvh_solve_packed_device(dvh_handle*, const dvh_packed*, void*) { return DVH_ERR_UNSUPPORTED; }
int dvh_warm_transfer(dvh_handle*, const dvh_packed*, const int32_t*, int32_t) { return DVH_ERR_UNSUPPORTED; }
int dvh_warm_transfer_blend(dvh_handle*, const dvh_packed*, const int32_t*, const double*, int32_t, int32_t) {
  return DVH_ERR_UNSUPPORTED;
}
int dvh_synchronize(dvh_handle*) { return DVH_OK; }
int dvh_last_stats(const dvh_handle*, int32_t* out4) {
  if (out4) std::memset(out4, 0, 4 * sizeof(int32_t));
  return DVH_OK;
}
int dvh_last_path_counts(const dvh_handle*, int32_t* out3) {
  if (out3) std::memset(out3, 0, 3 * sizeof(int32_t));
  return DVH_OK;
}
int dvh_last_path_counts4(const dvh_handle*, int32_t* out4) {
  if (out4) std::memset(out4, 0, 4 * sizeof(int32_t));
  return DVH_OK;
}
int dvh_build_battery_group(dvh_handle*, const dvh_battery_group*, const dvh_packed*, int32_t) {
  return DVH_ERR_UNSUPPORTED;  // device-only entry
}
int dvh_series_draws(dvh_handle*, const dvh_sweep_draws*) { return DVH_ERR_UNSUPPORTED; }       // device-only
int dvh_last_host_syncs(const dvh_handle*, int32_t* out) {
  if (out) *out = 0;  // no device stream
  return DVH_OK;
}
int dvh_series_windows(dvh_handle*, const dvh_window_series*) { return DVH_ERR_UNSUPPORTED; }   // device-only
int dvh_last_path_counts5(const dvh_handle*, int32_t* out5) {
  if (out5) std::memset(out5, 0, 5 * sizeof(int32_t));
  return DVH_OK;
}
int dvh_last_chain_aborts(const dvh_handle*, int32_t* out) {
  if (out) *out = 0;  // no team launches
  return DVH_OK;
}
const char* dvh_last_warning(const dvh_handle*) { return ""; }
int dvh_set_kernel_path(dvh_handle*, int) { return DVH_OK; }
int dvh_set_launch_order(dvh_handle*, const int32_t*, int32_t) { return DVH_OK; }
// the result all-gather is a device collective (RCCL): no communicator in the CPU restatement
int dvh_comm_unique_id(dvh_handle*, uint8_t*) { return DVH_ERR_UNSUPPORTED; }
int dvh_comm_init(dvh_handle*, int32_t, int32_t, const uint8_t*) { return DVH_ERR_UNSUPPORTED; }
int dvh_comm_info(const dvh_handle* h, int32_t* rw) {
  if (!h || !rw) return DVH_ERR_ARG;
  rw[0] = rw[1] = 0;
  return DVH_OK;
}
int dvh_gather_results(dvh_handle*, const void*, uint64_t, void*, void*) { return DVH_ERR_UNSUPPORTED; }
int dvh_outage_coverage(dvh_handle*, const dvh_outage_case*, int32_t, int32_t*, double*) { return DVH_ERR_UNSUPPORTED; }
int dvh_outage_min_soe(dvh_handle*, const dvh_outage_case*, int32_t, const int32_t*, double*) {
  return DVH_ERR_UNSUPPORTED;
}
int dvh_last_outage_ms(const dvh_handle*, double* ms) {
  if (ms) *ms = 0.0;
  return DVH_OK;
}

}  // extern "C"

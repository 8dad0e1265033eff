// dvh_build.hip -- device-side window builder: the battery + demand-charge + retail / DA window LP of
// dervet_hip/lp/builder.py battery_group, written straight into the packed batch in HBM.
//
// One 256-thread workgroup per window.  Every value is formed with the host builder's operations in the host
// builder's order (products as written there, the objective as the running sum of its terms in the terms
// dict's order), so the arrays are bit-identical to the host path (tests/test_gpu_builder.py); the CSR pattern is
// generated from (T, J, the demand-charge rows' steps and columns).  has_ice: the LP-relaxed ICE of battery_group's
// `ice` (columns elec_t, on_t after tau; the DCM rows gain elec_t; two >= rows per step after the DCM rows:
// cap on_t - elec_t >= 0, elec_t - pmin on_t >= 0; the fuel term last in the objective) -- BASELINE config 5.
#include <math.h>

#include "../../include/dervet_hip.h"
// Bit-identity with numpy needs every product rounded before it is added: no FMA contraction in this file.
#pragma clang fp contract(off)
#include "dvh_internal.h"

namespace dvh {
namespace {

constexpr int kBuildB = 256;

__global__ __launch_bounds__(kBuildB) void build_battery_kernel(const dvh_battery_group g, const int64_t* desc,
                                                               int32_t* indptr, int32_t* indices, double* data,
                                                               double* c, double* c0, double* q, double* l,
                                                               double* u, int first) {
  const int w = blockIdx.x;  // window within the group
  const int k = first + w;
  const int64_t* d = desc + 8 * (int64_t)k;
  const int T = g.T, J = g.J, mI = g.mI;
  const bool ice = g.has_ice != 0;
  const int n = (ice ? 5 : 3) * T + J, m = T + 1 + mI + (ice ? 2 * T : 0);
  const int CE = 3 * T + J, CO = 4 * T + J;  // first elec / on column (ICE)
  const int wd = ice ? 4 : 3;                 // entries per demand-charge row
  int32_t* ip = indptr + d[4];
  int32_t* ix = indices + d[5];
  double* dv = data + d[5];
  double* cv = c + d[6];
  double* lv = l + d[6];
  double* uv = u + d[6];
  double* qv = q + d[7];
  const int tid = threadIdx.x;
  const double dt = g.dt;
  const double E = g.E[w], eta = g.rte[w], sdr = g.sdr[w];
  const double target = g.soc_target[w] * E;
  const int fin = 1 + 4 * (T - 1);  // first entry of the end-of-window row
  const int dcm0 = fin + 3;         // first entry of the demand-charge rows
  const int ice0 = dcm0 + wd * mI;  // first entry of the ICE rows
  // ---- row pointers
  for (int r = tid; r <= m; r += kBuildB) {
    int v;
    if (r == 0) v = 0;
    else if (r <= T) v = 1 + 4 * (r - 1);
    else if (r <= T + 1 + mI) v = dcm0 + wd * (r - T - 1);
    else v = ice0 + 2 * (r - T - 1 - mI);
    ip[r] = v;
  }
  // ---- entries: row 0 (ene_0 = target), SOE rows (ch_t, dis_t, ene_t, ene_t+1), end row, demand-charge rows
  if (tid == 0) {
    ix[0] = 2 * T;
    dv[0] = 1.0;
    ix[fin] = T - 1;
    ix[fin + 1] = 2 * T - 1;
    ix[fin + 2] = 3 * T - 1;
    dv[fin] = dt * eta;
    dv[fin + 1] = -dt;
    dv[fin + 2] = 1.0 - dt * sdr;
  }
  const double a0 = -dt * eta, a2 = -(1.0 - dt * sdr);
  for (int t = tid; t < T - 1; t += kBuildB) {
    const int p = 1 + 4 * t;
    ix[p] = t;
    ix[p + 1] = T + t;
    ix[p + 2] = 2 * T + t;
    ix[p + 3] = 2 * T + t + 1;
    dv[p] = a0;
    dv[p + 1] = dt;
    dv[p + 2] = a2;
    dv[p + 3] = 1.0;
  }
  const double* base = g.base + (int64_t)w * T;
  for (int i = tid; i < mI; i += kBuildB) {
    const int p = dcm0 + wd * i, t = g.dcm_t[i];
    ix[p] = t;
    ix[p + 1] = T + t;
    ix[p + 2] = 3 * T + g.dcm_j[i];
    dv[p] = -1.0;
    dv[p + 1] = 1.0;
    dv[p + 2] = 1.0;
    if (ice) {
      ix[p + 3] = CE + t;
      dv[p + 3] = 1.0;
    }
    qv[T + 1 + i] = base[t];
  }
  if (ice) {  // per step: cap on_t - elec_t >= 0, elec_t - pmin on_t >= 0
    const double cap = g.ice_cap[w], pmin = g.ice_pmin[w];
    for (int t = tid; t < T; t += kBuildB) {
      const int p = ice0 + 4 * t;
      ix[p] = CE + t;
      ix[p + 1] = CO + t;
      ix[p + 2] = CE + t;
      ix[p + 3] = CO + t;
      dv[p] = -1.0;
      dv[p + 1] = cap;
      dv[p + 2] = 1.0;
      dv[p + 3] = -pmin;
      qv[T + 1 + mI + 2 * t] = 0.0;
      qv[T + 1 + mI + 2 * t + 1] = 0.0;
    }
  }
  // ---- right-hand side of the equality rows
  for (int r = tid; r <= T; r += kBuildB)
    if (r == 0 || r == T) qv[r] = target;
    else qv[r] = 0.0;
  // ---- bounds
  const double pch = g.pch[w], pdis = g.pdis[w];
  const double lo0 = g.llsoc[w] * E, hi0 = g.ulsoc[w] * E;
  const double* emin = g.has_emin ? g.emin + (int64_t)w * T : nullptr;
  const double* emax = g.has_emax ? g.emax + (int64_t)w * T : nullptr;
  for (int t = tid; t < T; t += kBuildB) {
    lv[t] = 0.0;
    uv[t] = pch;
    lv[T + t] = 0.0;
    uv[T + t] = pdis;
    double lo = lo0 * 1.0, hi = hi0 * 1.0;
    if (emin) lo = fmax(lo, emin[t]);
    if (emax) hi = fmin(hi, emax[t]);
    lv[2 * T + t] = lo;
    uv[2 * T + t] = hi;
  }
  for (int j = tid; j < J; j += kBuildB) {
    lv[3 * T + j] = -INFINITY;
    uv[3 * T + j] = INFINITY;
  }
  if (ice)
    for (int t = tid; t < T; t += kBuildB) {
      lv[CE + t] = 0.0;
      uv[CE + t] = INFINITY;
      lv[CO + t] = 0.0;
      uv[CO + t] = 1.0;
    }
  // ---- objective: the running sum of the terms in the host's dict order DA, DCM, retailETS, fixed_om, var_om
  // (, ICE fuel: zero on these columns)
  const double* da = g.has_da ? g.da + (int64_t)w * T : nullptr;
  const double* rt = g.has_retail ? g.retail + (int64_t)w * T : nullptr;
  const double varom = g.om[w] / 1000.0 * dt;
  for (int t = tid; t < T; t += kBuildB) {
    double ach = 0.0, adis = 0.0;
    if (da) {
      ach += da[t] * dt;
      adis += -da[t] * dt;
    }
    if (J) {
      ach += 0.0;
      adis += 0.0;
    }
    if (rt) {
      ach += rt[t] * dt;
      adis += -rt[t] * dt;
    }
    ach += 0.0;   // fixed_om
    adis += 0.0;
    ach += 0.0;   // var_om (dis only)
    adis += varom;
    if (ice) {
      ach += 0.0;
      adis += 0.0;
    }
    cv[t] = ach;
    cv[T + t] = adis;
    double aen = 0.0;
    if (da) aen += 0.0;
    if (J) aen += 0.0;
    if (rt) aen += 0.0;
    aen += 0.0;
    aen += 0.0;
    if (ice) aen += 0.0;
    cv[2 * T + t] = aen;
    if (ice) {  // elec_t reduces the net load like discharge; on_t has no cost
      double ael = 0.0, aon = 0.0;
      if (da) {
        ael += -da[t] * dt;
        aon += 0.0;
      }
      if (J) {
        ael += 0.0;
        aon += 0.0;
      }
      if (rt) {
        ael += -rt[t] * dt;
        aon += 0.0;
      }
      ael += 0.0;  // fixed_om
      aon += 0.0;
      ael += 0.0;  // var_om
      aon += 0.0;
      ael += g.ice_cost[w];
      aon += 0.0;
      cv[CE + t] = ael;
      cv[CO + t] = aon;
    }
  }
  for (int j = tid; j < J; j += kBuildB) {
    double a = 0.0;
    if (da) a += 0.0;
    a += g.demand[(int64_t)w * J + j];
    if (rt) a += 0.0;
    a += 0.0;
    a += 0.0;
    if (ice) a += 0.0;
    cv[3 * T + j] = a;
  }
  if (tid == 0) c0[k] = g.c0[w];
  (void)n;
}

}  // namespace

hipError_t launch_build_battery(const dvh_battery_group& g, const dvh_packed& b, int first, hipStream_t s) {
  hipLaunchKernelGGL(build_battery_kernel, dim3(g.G), dim3(kBuildB), 0, s, g, b.desc, const_cast<int32_t*>(b.indptr),
                     const_cast<int32_t*>(b.indices), const_cast<double*>(b.data), const_cast<double*>(b.c),
                     const_cast<double*>(b.c0), const_cast<double*>(b.q), const_cast<double*>(b.l),
                     const_cast<double*>(b.u), first);
  return hipGetLastError();
}

}  // namespace dvh

/*
 * dervet_hip.h -- C ABI of libdervet_hip, the MI355X batched dispatch-LP solver.
 *
 * Drop-in boundary.  In the reference every optimization window is solved by
 *   storagevet Scenario.solve_optimization(functions, constraints) -> (cvx_problem, obj_expressions, cvx_error_msg)
 * called once per window from the serial loop at dervet/MicrogridScenario.py:310-320 (optimize_problem_loop,
 * :281), i.e. CVXPY 1.0.31 canonicalisation + ECOS 2.0.7 / GLPK (cvxopt 1.2.5) in C (requirements.txt:1,2,5).
 * This library replaces that solve for LP windows: the caller exports every window's canonical LP
 *     min c'x + c0   s.t.  K_E x = q_E,  K_I x >= q_I,  l <= x <= u      (rows ordered E then I)
 * and solves all windows of all scenarios as ONE batch with a restarted reflected-Halpern PDHG
 * (PDLP family) in hand-written HIP for gfx950.  No pointers are retained after a call returns.
 *
 * Entry point  <->  reference interface it replaces
 *   dvh_create / dvh_destroy   : solver construction (cvx.Problem(...).solve(solver=...) picks ECOS/GLPK;
 *                                storagevet Scenario.solve_optimization, called at MicrogridScenario.py:319)
 *   dvh_solve_batch            : the per-window prob.solve() of MicrogridScenario.py:319, for `count`
 *                                windows at once (host buffers in / out)
 *   dvh_solve_packed_device    : same, on a batch already resident in HBM (bench / torch callers)
 *   dvh_last_error             : cvx_error_msg (errors travel as a message, MicrogridScenario.py:319-320)
 *   result.status              : maps to the cvxpy status strings read by save_optimization_results
 *                                (MicrogridScenario.py:348-363): OPTIMAL->"optimal",
 *                                PRIMAL_INFEASIBLE->"infeasible", DUAL_INFEASIBLE->"unbounded",
 *                                ITER_LIMIT->"optimal_inaccurate", NUMERICAL->"solver_error".
 *
 * Threading: one handle per host thread.  A handle drives every GPU whose bit is set in device_mask (0 = device 0):
 * dvh_solve_batch splits a host-buffer batch into contiguous ranges of near-equal estimated cost, one per device,
 * solved concurrently by one host thread per device (no inter-device traffic; each device writes its windows'
 * results straight into the caller's dvh_result buffers).  Device-resident batches (dvh_solve_packed_device) and
 * the reliability sweep run on the handle's first device.  Multi-process runs (one rank per GPU, torch.distributed
 * / RCCL all-gather of the results) use one single-device handle per rank.
 * Return codes: 0 = OK, negative = usage / HIP error (message via dvh_last_error).
 */
#ifndef DERVET_HIP_H
#define DERVET_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DVH_OK 0
#define DVH_ERR_ARG (-1)
#define DVH_ERR_HIP (-2)
#define DVH_ERR_UNSUPPORTED (-3)

/* per-window status */
#define DVH_OPTIMAL 0
#define DVH_PRIMAL_INFEASIBLE 1
#define DVH_DUAL_INFEASIBLE 2
#define DVH_ITER_LIMIT 3
#define DVH_NUMERICAL 4

/* structure hints (dvh_lp.structure) */
#define DVH_STRUCT_GENERIC_CSR 0
#define DVH_STRUCT_BATTERY_BANDED 1

typedef struct dvh_options {
  double eps;                 /* relative KKT tolerance (primal, dual, gap), default 1e-6          */
  int32_t max_iters;          /* per window, default 100000                                       */
  int32_t check_every;        /* restart-check period (iterations), default 32                    */
  int32_t ruiz_iters;         /* Ruiz equilibration passes, default 10                            */
  int32_t power_iters;        /* power-iteration steps for ||K||_2, default 64                    */
  double step_safety;         /* eta = step_safety / ||K||_2, default 0.998                       */
  double reflection;          /* Halpern reflection rho in [0,1], default 1                       */
  double restart_sufficient;  /* default 0.2  */
  double restart_necessary;   /* default 0.8  */
  double restart_artificial;  /* default 0.1  */
  double primal_weight_theta; /* default 1.0  */
  int32_t verbose;            /* 0 silent                                                           */
  int32_t kkt_every;          /* termination (KKT) check every kkt_every restart checks, default 4 */
  int32_t warm_start;         /* 1: start each window from the x / y already in the output buffers     */
                              /*    (unscaled, e.g. a similar window's solution); 0: x = proj(0), y = 0 */
  int32_t pad0;
  double eps_obj;             /* objective-error termination (0 = off), default 1e-6: besides the KKT test, */
                              /* |pobj - dobj| + ||y||_2 ||r_p||_2 <= eps_obj (1 + |pobj|) (unscaled), an    */
                              /* estimate of |pobj - opt| (gap + the dual-weighted primal residual)          */
  int32_t kkt_predict;        /* 0 = off (default).  P > 0 (band and ELL kernels; the other tiers ignore it): a  */
                              /* due KKT check is skipped while its predicted outcome, the last check's worst   */
                              /* ratio max(pres, dres, gap) / eps scaled by the fixed-point residual's decrease  */
                              /* since then, exceeds P; at most 4 due checks in a row are skipped.  Termination  */
                              /* still needs a KKT check that passes: this only saves hopeless checks.           */
  int32_t reserved;
} dvh_options;

typedef struct dvh_lp {
  int32_t n;                  /* variables                          */
  int32_t m_eq;               /* equality rows (first)              */
  int32_t m_ineq;             /* >= rows (after the equalities)     */
  int32_t nnz;
  const int32_t* indptr;      /* [m_eq + m_ineq + 1] CSR row pointers (0-based)                  */
  const int32_t* indices;     /* [nnz] column indices                                           */
  const double* data;         /* [nnz]                                                          */
  const double* c;            /* [n] objective                                                  */
  double c0;                  /* objective constant                                             */
  const double* q;            /* [m] right-hand side                                            */
  const double* l;            /* [n] lower bounds (-INFINITY allowed)                           */
  const double* u;            /* [n] upper bounds (+INFINITY allowed)                           */
  int32_t structure;          /* DVH_STRUCT_* hint (informational)                              */
  int32_t reserved;
} dvh_lp;

typedef struct dvh_result {
  double* x;                  /* caller-allocated [n] or NULL                                   */
  double* y;                  /* caller-allocated [m] or NULL (duals; >= rows have y >= 0)       */
  double obj;                 /* c'x + c0                                                       */
  double primal_res_rel;      /* ||(q - Kx)_proj||_2 / (1 + ||q||_2)                            */
  double dual_res_rel;        /* ||c - K'y - lambda||_2 / (1 + ||c||_2)                         */
  double gap_rel;             /* |pobj - dobj| / (1 + |pobj| + |dobj|)                          */
  int32_t status;             /* DVH_OPTIMAL ...                                                */
  int32_t iters;
} dvh_result;

/* A batch already resident in device memory ("packed" layout).
 * desc[8*k + 0..7] = {n, m, m_eq, nnz, off_row, off_nz, off_n, off_m} (int64) for window k:
 *   indptr[off_row .. off_row+m]   (window-local row pointers, int32)
 *   indices/data[off_nz .. +nnz]   (window-local column indices int32 / values f64)
 *   c,l,u[off_n .. +n], q[off_m .. +m], c0[k]
 * Outputs: x[off_n..], y[off_m..], stats[4k..4k+3] = {obj, primal_res_rel, dual_res_rel, gap_rel},
 *          istats[2k..2k+1] = {status, iters}.  All pointers are device pointers. */
typedef struct dvh_packed {
  int32_t count;
  int32_t reserved;
  int64_t total_n, total_m, total_nnz, total_rows; /* sizes of the concatenated arrays (rows = sum(m+1)) */
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
} dvh_packed;

typedef struct dvh_handle dvh_handle;

const char* dvh_version(void);
void dvh_default_options(dvh_options* opts);
int dvh_create(int device_mask, const dvh_options* opts, dvh_handle** out);
/* The same with an explicit device list (devices may repeat: several concurrent sub-handles on one GPU). */
int dvh_create_devices(const int32_t* devices, int32_t n, const dvh_options* opts, dvh_handle** out);
/* Devices (sub-handles) of a handle. */
int dvh_device_count(const dvh_handle* h);
int dvh_destroy(dvh_handle* h);
const char* dvh_last_error(const dvh_handle* h);
int dvh_set_options(dvh_handle* h, const dvh_options* opts);

/* ---- The result all-gather across ranks.  One process per GPU: the windows are sharded over the
 * ranks with no traffic during the solve, then ONE all-gather returns every window's result row (objective,
 * residuals, status, iterations, (scenario, window) tag, dispatch) to every rank.  Replaces the reference's serial
 * case loop (dervet/DERVET.py:75-83).  RCCL is opened at run time (librccl.so.1 of /opt/rocm, or DVH_RCCL_LIB);
 * DVH_ERR_UNSUPPORTED when it cannot be.
 *   dvh_comm_unique_id: rank 0 draws the 128-byte id (ncclGetUniqueId) the launcher hands to every rank;
 *   dvh_comm_init: joins rank `rank` of `world` on the handle's device (single-device handles only);
 *   dvh_comm_info: {rank, world} (0, 0 without a communicator);
 *   dvh_gather_results: out[world * bytes_per_rank] (device) = every rank's rows[bytes_per_rank] (device) in rank
 *     order; asynchronous on `stream` (a hipStream_t; NULL = the handle's solver stream, i.e. after its solves). */
#define DVH_COMM_ID_BYTES 128
int dvh_comm_unique_id(dvh_handle* h, uint8_t* id);
int dvh_comm_init(dvh_handle* h, int32_t rank, int32_t world, const uint8_t* id);
int dvh_comm_info(const dvh_handle* h, int32_t* rank_world);
int dvh_gather_results(dvh_handle* h, const void* rows, uint64_t bytes_per_rank, void* out, void* stream);

/* Host buffers in / out.  Blocks until the batch is solved. */
int dvh_solve_batch(dvh_handle* h, const dvh_lp* lps, int32_t count, dvh_result* out);

/* Device-resident batch; `stream` is a hipStream_t (NULL = the handle's own stream).  Asynchronous
 * w.r.t. the host when stream != NULL; call dvh_synchronize / hipStreamSynchronize before reading. */
int dvh_solve_packed_device(dvh_handle* h, const dvh_packed* batch, void* stream);

/* ---- Device-side window builder (the LP that storagevet's
 * set_up_optimization builds for a battery + demand-charge + retail / DA window, MicrogridScenario.py:322-346).
 * Expands G windows' inputs (device pointers) into the packed batch's LP arrays, windows first .. first + G - 1,
 * whose descriptors the caller has set (n = 3T + J, m = T + 1 + mI, nnz = 4T + 3 mI, any offsets; ICE below).  The values are
 * exactly those of dervet_hip/lp/builder.py battery_group (same formulas, same summation order; bit-identical,
 * tests/test_gpu_builder.py), so a sweep ships its compact inputs to HBM instead of the expanded LPs.
 * Asynchronous on the handle's stream. */
typedef struct dvh_battery_group {
  int32_t T, J, G, mI;             /* steps, demand-charge (tau) columns, windows, demand-charge rows           */
  double dt;                       /* hours per step                                                             */
  int32_t has_retail, has_da;      /* price inputs present                                                       */
  int32_t has_emin, has_emax;      /* aggregate-SOE limits present                                               */
  const int32_t* dcm_t;            /* [mI] step of each demand-charge row (rows in builder order)                */
  const int32_t* dcm_j;            /* [mI] its tau column                                                        */
  const double* base;              /* [G*T] net load + housekeeping power, kW (load - fixed PV + hp)             */
  const double* retail;            /* [G*T] $/kWh or NULL                                                        */
  const double* da;                /* [G*T] $/kWh or NULL                                                        */
  const double* demand;            /* [G*J] $/kW                                                                 */
  const double* emin;              /* [G*T] kWh or NULL                                                          */
  const double* emax;              /* [G*T] kWh or NULL                                                          */
  const double* E;                 /* [G] energy capacity, kWh                                                   */
  const double* pch;               /* [G] kW                                                                     */
  const double* pdis;              /* [G] kW                                                                     */
  const double* rte;               /* [G] round-trip efficiency, fraction                                        */
  const double* sdr;               /* [G] self-discharge, fraction per hour (sdr % / 100)                        */
  const double* soc_target;        /* [G] fraction                                                               */
  const double* ulsoc;             /* [G] fraction                                                               */
  const double* llsoc;             /* [G] fraction                                                               */
  const double* om;                /* [G] variable O&M, $/MWh                                                    */
  const double* c0;                /* [G] objective constant (the terms' constants, summed on the host)          */
  /* LP-relaxed ICE (BASELINE config 5; builder.battery_group `ice`): columns elec_t, on_t after tau (n = 5T + J),
   * elec_t in every demand-charge row (4 entries), two >= rows per step after them (m = 3T + 1 + mI,
   * nnz = 8T + 4 mI): cap on_t - elec_t >= 0, elec_t - pmin on_t >= 0; elec in [0, inf), on in [0, 1].  */
  int32_t has_ice, pad_ice;
  const double* ice_cap;           /* [G] rated power x units, kW                                                */
  const double* ice_pmin;          /* [G] minimum stable power x units, kW                                       */
  const double* ice_cost;          /* [G] (efficiency x fuel cost + variable O&M) x dt, $/kW per step             */
} dvh_battery_group;
int dvh_build_battery_group(dvh_handle* h, const dvh_battery_group* group, const dvh_packed* batch, int32_t first);
int dvh_synchronize(dvh_handle* h);

/* ---- Synthetic scenario series on the device (BASELINE.json configs 4 / 5; no reference
 * counterpart: the reference reads one time-series CSV per case, dervet/DERVET.py:75-83, and a sweep's perturbed
 * series are this framework's workload generator, dervet_hip/lp/scenarios.py).  Draws, per scenario, exactly what
 * numpy's np.random.Generator(np.random.PCG64(seed)) draws on the host: one standard normal (the lognormal load
 * scale), `steps` standard normals filtered as scipy.signal.lfilter([1], [1, a1]) with the innovations after the
 * first scaled by `innov`, then `n_uniform` next_double words (uniform(low, high) = low + (high - low) * u).
 * seeds: host [count] SeedSequence entropy; z0 [count], ar [count * steps], uniform [count * n_uniform]: device.
 * Bit-identical to the host generator (tests/test_gpu_series.py).  DVH_ERR_UNSUPPORTED if a wedge test of the
 * ziggurat fell within 2^-40 of the device exp (its outcome could differ from the host libm's; not observed).
 * Returns after the kernel completed. */
typedef struct dvh_sweep_draws {
  int32_t count, steps, n_uniform;
  const uint64_t* seeds;
  double a1;                       /* lfilter denominator coefficient a[1] (-phi)                              */
  double innov;                    /* innovation scale of steps >= 1 (sqrt(1 - phi^2))                         */
  double* z0;
  double* ar;
  double* uniform;
  /* optional [count] int32 (device): 1 for a scenario whose ziggurat wedge test landed within 2^-40 of exp() (its
   * draws may differ from numpy's), else 0.  Given, such scenarios are only flagged (the caller regenerates them on
   * the host) and the call returns DVH_OK; NULL: any such scenario fails the call with DVH_ERR_UNSUPPORTED. */
  int32_t* ambiguous;
} dvh_sweep_draws;
int dvh_series_draws(dvh_handle* h, const dvh_sweep_draws* d);

/* The device builder's inputs (dvh_battery_group base / retail / c0) of G windows cut from the scenarios' series:
 * window k of scenario rows[k] covers steps t0 .. t0 + T - 1 (rep steps per hour of the hourly series);
 *   base[k][t]   = (site_load[h] * load_scale[s]) * (1 + 0.05 * ar[s][h]) - pv_rated[s] * pv_profile[h] + hp[s],
 *   retail[k][t] = price[t0 + t] * price_scale[s],                                  h = (t0 + t) / rep,
 *   c0[k]        = the retail term's constant sum((retail * dt) * base) as numpy sums it (in step order; pairwise
 *                  when G = 1), + c0_add[s]
 * (J > 0: the window has demand-charge columns, which add zero constants).  All pointers device; rows are
 * range-checked on the device (DVH_ERR_ARG).  Asynchronous on the handle's stream; returns after it completed. */
typedef struct dvh_window_series {
  int32_t G, T, t0, rep, J, count, hours;
  double dt;
  const int32_t* rows;             /* [G] scenario of each window, 0 <= rows[k] < count                        */
  const double* ar;                /* [count * hours] (dvh_series_draws)                                       */
  const double* site_load;         /* [hours] kW                                                                */
  const double* pv_profile;        /* [hours] kW per rated kW (NaN as 0)                                        */
  const double* price;             /* [>= t0 + T] energy price per step, $/kWh                                  */
  const double* load_scale;        /* [count]                                                                   */
  const double* price_scale;       /* [count]                                                                   */
  const double* pv_rated;          /* [count] kW                                                                */
  const double* hp;                /* [count] housekeeping power, kW                                            */
  const double* c0_add;            /* [count] fixed O&M x discharge rating                                      */
  double* base;                    /* out [G * T]                                                               */
  double* retail;                  /* out [G * T]                                                               */
  double* c0;                      /* out [G]                                                                   */
} dvh_window_series;
int dvh_series_windows(dvh_handle* h, const dvh_window_series* w);

/* ---- Seeded scenario sweeps (dervet_hip/sweep.py; the sensitivity cases of dervet/DERVET.py:75 solve the same
 * windows for many perturbed scenarios; no reference counterpart: the reference solves every window cold).
 * Warm starts for `count` windows of a device-resident packed batch from solved partner windows of the same LP
 * shape, in one launch on the handle's stream (ordered with the solves; returns after it completed).
 * pairs (host, int32 [count][3]): {window, partner window, T}.  x <- the partner's x scaled per column by
 * u_window / u_partner where both are finite and u_partner > 0, else copied; T > 0 (battery + DCM shape,
 * n = 3T + 1): the duals of rows 0..T scaled by mean|c_window[0:T]| / mean|c_partner[0:T]| and the others by
 * c_window[3T] / c_partner[3T] (denominators clamped at 1e-12); T <= 0: duals copied.  DVH_ERR_ARG for a pair
 * naming no window, a window listed twice, a partner that is itself listed (checked before the launch), or windows
 * of different shape (those pairs are skipped, the others applied). */
int dvh_warm_transfer(dvh_handle* h, const dvh_packed* batch, const int32_t* pairs, int32_t count);
/* The same from a weighted blend of q partners (1 <= q <= 8): rows[count][q + 2] = {window, partner_1 .. partner_q, T},
 * weights[count][q] (host; normally summing to 1): x = sum_k w_k x_k', y = sum_k w_k y_k' with x_k', y_k' partner k's
 * solution transferred as dvh_warm_transfer does (summed in row order).  q = 1 with weight 1 is dvh_warm_transfer bit
 * for bit.  DVH_ERR_ARG as dvh_warm_transfer, and for q out of range or a weight that is not finite. */
int dvh_warm_transfer_blend(dvh_handle* h, const dvh_packed* batch, const int32_t* rows, const double* weights,
                            int32_t count, int32_t q);

/* Timing of the most recent solve on the handle's stream (HIP events, milliseconds):
 * [0] whole solve, [1] setup kernel (transpose + scaling + power iteration), [2] PDHG kernels.  On the default
 * cascade the band kernels scale the windows they take themselves, inside the PDHG launch, and the setup kernel runs
 * only for what they refuse, between the cascade's PDHG launches: there [1] is ~0 and [2] holds all of it (setup
 * included); the A/B paths (dvh_set_kernel_path 1 / 2) run setup_kernel first and split the two as written. */
int dvh_last_timing(const dvh_handle* h, double* ms3);

/* Host waits on the stream during the most recent solve (dvh_solve_batch / dvh_solve_packed_device): the
 * descriptors' read-back (device batches), one per kernel tier that ran (the cascade's lists are formed on the
 * device, dvh_route.hip), the medium tier's hand-offs, and the final wait for the results and timing events. */
int dvh_last_host_syncs(const dvh_handle* h, int32_t* out);
/* Kernel-path diagnostics of the most recent solve: out4 = {windows solved by the ELL fast kernel,
 * windows solved by the generic CSR kernel, kernel variant code, generic_only flag}. */
int dvh_last_stats(const dvh_handle* h, int32_t* out4);
/* Windows per solver path in the most recent solve: out3 = {ELL kernel, generic CSR kernel, grid-wide
 * large-LP path (n or m > 4096: one window at a time over the whole GPU, e.g. BASELINE config 3)}. */
int dvh_last_path_counts(const dvh_handle* h, int32_t* out3);
/* The same plus the battery-banded kernel: out4 = {ELL kernel, generic CSR kernel, grid-wide large-LP path,
 * battery-banded kernel (windows with the storagevet battery + DCM structure, detected on the device)}. */
int dvh_last_path_counts4(const dvh_handle* h, int32_t* out4);
/* The same plus the medium tier: out5 = {ELL, generic, grid-wide, battery-banded, medium tier (battery windows of
 * 769 .. 12,288 steps -- the annual hourly window n = "year", sub-hourly monthly windows -- solved as a batch, a
 * team of one workgroup per <= 768-step segment per window, dvh_chain.hip)}. */
int dvh_last_path_counts5(const dvh_handle* h, int32_t* out5);
/* Medium-tier team launches of the most recent solve that aborted (a segment exchange outlasted the spin limit): the
 * windows such a launch had finished keep their results, the others were solved on the grid-wide path, and the solve
 * still returns DVH_OK.  out = that count (0 when nothing aborted); reset by every solve. */
int dvh_last_chain_aborts(const dvh_handle* h, int32_t* out);
/* Diagnostics of a successful solve that took a fallback (a medium-tier abort: the workgroups' exchange state), or
 * "" -- dvh_last_error is left to errors.  Reset by every solve. */
const char* dvh_last_warning(const dvh_handle* h);
/* ---- Post-facto reliability sweep.
 * Replaces Reliability.load_coverage_probability (dervet/MicrogridValueStreams/Reliability.py:876-967) and the
 * serial recursion it drives (data_process :447-487, simulate_outage :489-570): for every case, an outage is
 * simulated from EVERY start step (one GPU thread each) and the covered lengths give the load coverage
 * probability curve P(outage of L hours covered), L = dt, 2 dt, .., max_outage.  The DER aggregates are the
 * caller's (Reliability.get_der_mix_properties :276-332): pv_vari = sum of pv_max x nu, gamma = largest gamma,
 * dg_gen = total ICE power (minus the largest unit for N-2), ESS limits = llsoc / ulsoc x energy rating. */
typedef struct dvh_outage_case {
  int32_t n_steps;                /* len(critical load)                                              */
  int32_t max_outage;             /* max_outage_duration (hours; also the data window in steps, :462) */
  double dt;                      /* hours per step                                                  */
  const double* critical_load;    /* [n_steps] kW                                                    */
  const double* pv_max;           /* [n_steps] total PV maximum generation, or NULL (no PV)          */
  const double* pv_vari;          /* [n_steps] total PV generation x nu, or NULL (no PV)             */
  const double* init_soe;         /* [n_steps] ESS energy at each outage start, or NULL: soe0        */
  const double* load_shed_pct;    /* [max_outage] % of the critical load kept per outage hour, or NULL */
  double soe0;                    /* energy at every start when init_soe == NULL (soc_init x rating) */
  double dg_gen;                  /* total generator power, kW (constant)                            */
  double gamma;                   /* largest PV gamma (fraction)                                     */
  double soe_min, soe_max;        /* ESS operation energy limits, kWh                                */
  double charge_max, discharge_max; /* kW                                                            */
  double rte;                     /* round-trip efficiency (fraction)                                */
} dvh_outage_case;

/* lengths: caller-allocated [sum n_steps] covered steps per start (case-major), or NULL;
 * lcp: caller-allocated [sum int(max_outage / dt)] load coverage probability per outage length.
 * Bit-exact with the reference's numpy arithmetic.  Blocks until done. */
int dvh_outage_coverage(dvh_handle* h, const dvh_outage_case* cases, int32_t count, int32_t* lengths,
                        double* lcp);
/* Reliability minimum-SOE requirement (Reliability.min_soe_iterative, Reliability.py:685-756, which feeds the
 * 'energy' 'min' system requirement of every window, :334-354): for every start step, an outage of
 * target_hours[k] (the Reliability 'target') simulated from soe0 (= soc_init x energy rating; init_soe and
 * load_shed_pct as above, init_soe ignored); min_soe[start] = max - min of its SOE profile including the start.
 * min_soe: caller-allocated [sum n_steps] (case-major).  Bit-exact with the numpy reference. */
int dvh_outage_min_soe(dvh_handle* h, const dvh_outage_case* cases, int32_t count, const int32_t* target_hours,
                       double* min_soe);
/* Kernel time of the last dvh_outage_coverage / dvh_outage_min_soe call (HIP events, milliseconds). */
int dvh_last_outage_ms(const dvh_handle* h, double* ms);

/* Kernel cascade (testing / A-B timing): 0 = default (battery-banded -> ELL -> generic CSR), 1 = generic
 * CSR kernel for every window, 2 = ELL -> generic (no battery-banded kernel), 3 / 4 = as 0 with the battery-banded
 * kernel's form forced: one step per lane (768 threads per window, one window per CU) / three steps per lane (256
 * threads, two windows per CU).  The default picks the one-step form when the batch has at most one battery window
 * per compute unit, else the three-step form. */
int dvh_set_kernel_path(dvh_handle* h, int mode);

/* Launch order of the next solve (scheduling only: the results do not depend on it).  order: host array, a
 * permutation of 0 .. count - 1 (validated; DVH_ERR_ARG otherwise), copied.  The next dvh_solve_packed_device /
 * dvh_solve_batch launches its battery-band pass over the windows in this order when count equals its window count
 * and the batch is one chunk of on-chip windows (else the packing order); the order is consumed by that solve.
 * Longest-expected-first orders shorten the launch's tail (dervet_hip/sweep.py orders a warm phase by its seeds'
 * iteration counts).  count 0 clears. */
int dvh_set_launch_order(dvh_handle* h, const int32_t* order, int32_t count);

#ifdef __cplusplus
}
#endif
#endif /* DERVET_HIP_H */

"""ORACLE (test infrastructure only; never shipped or measured): restatement of DER-VET's post-facto
reliability sweep, the load-coverage-probability curve.

Follows dervet/MicrogridValueStreams/Reliability.py, line by line in semantics:
  * load_coverage_probability  :876-967   one outage simulated from EVERY start step, a histogram of the
                                          covered lengths, P(covered >= L) = sum(freq[L/dt:]) / (N - L/dt + 1)
  * data_process               :447-487   demand_left / reliability_check rounded to 5 decimals, energy check
                                          = reliability_check * largest_gamma, optional load-shed multipliers
  * simulate_outage            :489-570   the recursion, written as a loop: charge from excess generation
                                          into the ESS, else discharge to cover the load (checks rounded to 2
                                          decimals); the outage is covered up to the first step that fails
  * get_der_mix_properties     :276-332   DER aggregates (pv_max, pv_max * nu, largest gamma, DG power)
  * min_soe_iterative          :685-756   minimum SOE per start = max - min of the SOE profile of a
                                          target-length outage (the config-5 reliability requirement, a10)
Rounding is numpy's ``around`` (x * 10**d, round half to even, / 10**d), restated with Python floats.
Pinned against the reference's golden ``load_coverage_prob*.csv`` curves (tests/test_outage_oracle.py).
"""
import numpy as np


def _around(x, f):
    """numpy.around(x, decimals=d) for a Python float, f = 10.0 ** d (multiply, round-half-even, divide)."""
    return round(x * f) / f


def data_arrays(critical_load, pv_max=None, nu=1.0, dg_gen=0.0, load_shed_pct=None):
    """Per-step inputs of data_process for the whole series: critical load, dg generation (constant),
    pv_max and pv_vari = pv_max * nu (Reliability.py:305-311)."""
    cl = np.asarray(critical_load, np.float64)
    N = len(cl)
    pmax = np.zeros(N) if pv_max is None else np.asarray(pv_max, np.float64)
    pvar = pmax * nu
    gen = np.repeat(float(dg_gen), N)
    return cl, gen, pmax, pvar


def simulate_outage(t, cl, gen, pmax, pvar, gamma, ess, init_soe, outage_len, max_steps, dt, load_shed_pct=None):
    """Covered length (steps) of the outage starting at step t, and its SOE profile (Reliability.py:489-570).

    ess: dict with 'charge max', 'discharge max', 'operation SOE min', 'operation SOE max', 'rte'."""
    N = len(cl)
    stop = min(t + max_steps, N)  # data_process slices max_steps entries (Reliability.py:462-465)
    ls = None
    if load_shed_pct is not None:
        ls = [v / 100.0 for v in load_shed_pct]
    soe = float(init_soe)
    prof = []
    for k in range(outage_len):
        i = t + k
        if i >= stop:  # no data left (Reliability.py:524)
            break
        c = float(cl[i])
        if ls is not None:
            c = c * ls[k]
        dl = _around(c - float(gen[i]) - float(pmax[i]), 1e5)
        rc = _around(c - float(gen[i]) - float(pvar[i]), 1e5)
        ec = rc * gamma
        if 0 >= rc:  # excess generation: charge if there is room (Reliability.py:529-541)
            emax = ess["operation SOE max"]
            if emax >= soe:
                rte = ess["rte"]
                charge_possible = (emax - soe) / (rte * dt)
                charge = min(charge_possible, -dl, ess["charge max"])
                soe = soe + (charge * rte * dt)
        else:  # discharge to cover the load (Reliability.py:544-564)
            emin = ess["operation SOE min"]
            if 0 >= _around(ec * dt - soe, 1e2):
                discharge_possible = (soe - emin) / dt
                discharge = min(discharge_possible, dl, ess["discharge max"])
                if 0 < _around(dl - discharge, 1e2):
                    break
                soe = soe - (discharge * dt)
            else:
                break
        prof.append(soe)
    return len(prof), prof


def coverage_lengths(cl, gen, pmax, pvar, gamma, ess, init_soe, max_outage_duration, dt, load_shed_pct=None):
    """Covered length for an outage starting at every step (Reliability.py:920-945). init_soe: [N] or scalar."""
    N = len(cl)
    outage_len = int(max_outage_duration / dt)
    soe0 = np.broadcast_to(np.asarray(init_soe, np.float64), (N,))
    out = np.zeros(N, np.int32)
    for t in range(N):
        out[t], _ = simulate_outage(t, cl, gen, pmax, pvar, gamma, ess, soe0[t], outage_len,
                                    int(max_outage_duration), dt, load_shed_pct)
    return out


def min_soe(cl, gen, pmax, pvar, gamma, ess, soc_init, outage_duration, max_outage_duration, dt,
            load_shed_pct=None):
    """Reliability.min_soe_iterative (Reliability.py:685-733): for every start, simulate an outage of
    outage_duration / dt steps from soc_init x energy rating and return soe_used (:734-756) = max - min of the
    SOE profile including the starting SOE.  [N] array (the 'Reliability Min State of Energy (kWh)')."""
    N = len(cl)
    soe0 = soc_init * ess["energy rating"]
    out = np.zeros(N)
    for t in range(N):
        _, prof = simulate_outage(t, cl, gen, pmax, pvar, gamma, ess, soe0, int(outage_duration / dt),
                                  int(max_outage_duration), dt, load_shed_pct)
        prof.insert(0, soe0)
        out[t] = np.max(prof) - np.min(prof)
    return out


def lcp_curve(lengths, max_outage_duration, dt):
    """Load coverage probability per outage length dt, 2 dt, .., max (Reliability.py:947-957)."""
    N = len(lengths)
    outage_len = int(max_outage_duration / dt)
    freq = np.bincount(np.asarray(lengths), minlength=outage_len + 1).astype(np.float64)
    out = []
    length = dt
    while length <= max_outage_duration:
        covered = freq[int(length / dt):].sum()
        total = N - (length / dt) + 1
        with np.errstate(divide="ignore", invalid="ignore"):  # N < L: the reference divides by <= 0 too
            out.append(np.float64(covered) / np.float64(total))
        length += dt
    return np.array(out)


def ess_props(E, P_ch, P_dis, rte, llsoc=0.0, ulsoc=1.0):
    """get_der_mix_properties for one ESS (Reliability.py:318-329; storagevet operational_min/max_energy =
    llsoc / ulsoc x energy capacity)."""
    return {"charge max": float(P_ch), "discharge max": float(P_dis), "operation SOE min": llsoc * float(E),
            "operation SOE max": ulsoc * float(E), "rte": float(rte), "energy rating": float(E)}

"""ORACLE (test infrastructure only): the battery benefit and the CBA present values the window results feed.

DER-VET's consumers of the solved windows: the monthly bill with / without the DERs
(storagevet Financial, absent here; its output simple_monthly_bill*.csv is golden), the pro forma that carries
each year's avoided charges (dervet/CBA.py:299-346 proforma_report, on storagevet Financial) and its NPV row
(dervet/CBA.py:212 annuity_scalar and storagevet's npv report use numpy's ``np.npv``, removed from numpy >= 1.20,
restated below).  Restated only as far as the goldens pin them:

  * original charges: the window's retail energy charge and demand charges of the site load alone
    (no battery, no PV): reproduces every "Original Energy / Demand Charge ($)" of the Usecase 2 golden bills
    (tests/test_benefit.py);
  * battery benefit of a window = original - (retailETS + DCM of the solved window): per window it equals the
    golden "Original - Energy / Demand Charge" difference, and the 12 monthly benefits of the opt year sum to the
    golden pro forma's "Avoided Energy / Demand Charge" of 2017;
  * later years escalate the opt year's avoided charge by the value stream's growth rate (retailTimeShift /
    DCM ``growth``, 2.2 %/yr in the goldens): the golden pro forma rows 2018-2037 are exactly that;
  * NPV = sum_k v_k / (1 + r)^k with k = 0 at the CAPEX row (numpy's npv): reproduces the golden npv row.
"""
import numpy as np


def npv(rate, values):
    """numpy.npv (numpy < 1.20 / numpy-financial): sum_k values[k] / (1 + rate)^k, k = 0, 1, ..."""
    v = np.asarray(values, np.float64)
    return float(np.sum(v / (1.0 + rate) ** np.arange(len(v))))


def original_charges(win):
    """(energy, demand) charge of a window's site load alone (the golden "Original ... Charge" columns)."""
    L = np.asarray(win["load"], np.float64)
    energy = float(np.sum(np.asarray(win["retail_price"], np.float64) * L * float(win["dt"])))
    demand = float(sum(d * L[np.asarray(m, bool)].max() for d, m in win["demand"]))
    return energy, demand


def no_battery_objective(lp):
    """Objective of a battery (+ DCM) window LP (oracle.window_lp / builder layout x = [ch, dis, ene, tau]) with
    the battery idle: ch = dis = 0 and each tau_j at the largest right-hand side of its DCM rows, i.e. the
    window's cost without the battery's dispatch (c0 keeps its constants).  obj - no_battery_objective is minus
    the battery benefit."""
    K = lp["K"].tocsr()
    q, c, me = np.asarray(lp["q"]), np.asarray(lp["c"]), int(lp["m_eq"])
    T = me - 1
    tau = {}
    for i in range(me, K.shape[0]):
        cols = K.indices[K.indptr[i]:K.indptr[i + 1]]
        tj = [j for j in cols if j >= 3 * T]
        if len(tj) != 1:
            raise ValueError("not a battery + DCM window")
        tau[tj[0]] = max(tau.get(tj[0], -np.inf), q[i])
    return float(lp["c0"] + sum(c[j] * v for j, v in tau.items()))


def escalate(v0, growth_pct, years):
    """Year-by-year values from the opt year's value and a growth rate in %/yr (years = number of years)."""
    return float(v0) * (1.0 + growth_pct / 100.0) ** np.arange(years)


def proforma_npv(bills, avoided_energy0=None, avoided_demand0=None):
    """NPV of the golden pro forma (dict from tests/golden/uc2_bills.json), optionally with its avoided-charge
    columns rebuilt from opt-year values: returns {column: npv, "Lifetime Present Value": npv of the yearly net}."""
    pf = {k: np.asarray(v, np.float64) for k, v in bills["proforma"].items()}
    rate = bills["npv_discount_rate"] / 100.0
    years = len(bills["proforma_index"]) - 1          # the rows after "CAPEX Year"
    for col, v0, key in (("Avoided Energy Charge", avoided_energy0, "retailTimeShift"),
                         ("Avoided Demand Charge", avoided_demand0, "DCM")):
        if v0 is not None:
            new = np.concatenate([[0.0], escalate(v0, bills["growth"][key], years)])
            pf["Yearly Net Value"] = pf["Yearly Net Value"] - pf[col] + new
            pf[col] = new
    out = {k: npv(rate, v) for k, v in pf.items() if k != "Yearly Net Value"}
    out["Lifetime Present Value"] = npv(rate, pf["Yearly Net Value"])
    return out

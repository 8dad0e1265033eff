"""The degradation restatement (dervet_hip/degradation.py) on the reference's own degradation cases, solved by the
oracle (restated LP + HiGHS) -- the CPU leg; tests/test_gpu_degradation_ref.py runs the same cases through the GPU.

What the reference asserts on these inputs (the only pins the absent storagevet degradation module has):
  * 040-Degradation_Test_MP.csv (test_2finances.py:44-75): the 2017 avoided energy charge is above 2022's, and the
    years after the last opt year equal 2022's (retailTimeShift growth 0);
  * 041-no_Degradation_Test_MP.csv (:78-104): yearly_degrade 10 but incl_cycle_degrade 0 -- the 2017 and 2022
    avoided energy charges are EQUAL, i.e. the module is off as a whole (dervet gates it on incl_cycle_degrade,
    Battery.py:82, :101);
  * 010-degradation_test.csv (test_3battery.py:74-75, "battery replaced during optimization"): the case runs.  It is
    not replaceable (replaceable 0), so the capacity may only shrink; the restatement records whether and when it
    reaches its state of health (Battery.py:102-104).
"""
import numpy as np
import pytest

from oracle import cba

import degradation_ref as dr


@pytest.fixture(scope="module")
def runs():
    out = {}
    for name, case in dr.cases().items():
        sw, build = dr.sweep(case)
        res = sw.run(dr.HighsSolver(), device=None)
        out[name] = (case, sw, build, res)
    return out


def test_fixture_is_the_reference_cases(runs):
    c = dr.cases()
    assert c["040"]["battery"]["incl_cycle_degrade"] == "1" and c["041"]["battery"]["incl_cycle_degrade"] == "0"
    assert c["040"]["battery"]["yearly_degrade"] == c["041"]["battery"]["yearly_degrade"] == "10"
    assert dr.opt_years(c["040"]) == [2017, 2022] and c["010"]["battery"]["replaceable"] == "0"


def test_040_older_opt_year_saves_more_and_later_years_are_flat(runs):
    case, sw, build, res = runs["040"]
    assert all((p["status"] == 0).all() for p in res)
    caps = np.array([p["capacity_before"][0] for p in res])
    assert (np.diff(caps) < 0).all()                      # calendar 10 %/yr + cycling, every window
    av = dr.avoided_charges(case, sw, build, res)
    assert av[2017] > av[2022] > 0.0                      # test_2finances.py:67-69
    growth = float(case["value_streams"]["retailTimeShift"]["growth"])
    later = cba.escalate(av[2022], growth, 2030 - 2022 + 1)[1:]
    assert np.all(later / av[2022] == 1.0)                # test_2finances.py:71-75


def test_041_no_cycle_degradation_means_no_degradation(runs):
    case, sw, build, res = runs["041"]
    caps = np.array([p["capacity_before"][0] for p in res])
    assert (caps == float(case["battery"]["ene_max_rated"])).all() and sw.deg.degrade_perc[0] == 0.0
    av = dr.avoided_charges(case, sw, build, res)
    assert av[2017] == av[2022]                           # test_2finances.py:102-104 (exact)


def test_010_runs_and_a_non_replaceable_battery_only_wears(runs):
    case, sw, build, res = runs["010"]
    assert all((p["status"] == 0).all() for p in res)
    caps = np.array([p["capacity_before"][0] for p in res])
    assert (np.diff(caps) <= 0).all() and sw.deg.replacements[0] == 0
    assert sw.deg.capacity()[0] < float(case["battery"]["ene_max_rated"])

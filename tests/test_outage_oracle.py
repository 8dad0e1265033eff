"""The reliability-sweep oracle (oracle/outage.py) reproduces the reference's golden load-coverage-probability
curves exactly: 3 post-facto runs of test_validation_report_sept1/Results/Usecase2/*/step2 (SOE from the
results, with and without PV) and the 2 load-shedding runs of test/test_load_shedding (soc_init x rating, with
and without load-shed multipliers)."""
import numpy as np
import pytest

import outage_cases


CASES = outage_cases.load()


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_golden_lcp(name):
    c = CASES[name]
    _, lcp = outage_cases.oracle_curve(c)
    assert lcp.shape == c["golden_lcp"].shape
    np.testing.assert_array_equal(lcp, c["golden_lcp"])


def test_der_mix_properties_restates_reference():
    """Host-side DER aggregation of dervet_hip.reliability (Reliability.get_der_mix_properties :276-332)."""
    from dervet_hip.reliability import OutageCase, der_mix_properties
    N = 48
    g1, g2 = np.linspace(0, 100, N), np.linspace(50, 0, N)
    c = OutageCase(critical_load=np.ones(N), ess=dict(E=100.0, P_ch=20.0, P_dis=25.0, rte=0.9, llsoc=0.1, ulsoc=0.95),
                   pv_max=[g1, g2], pv_nu=[0.2, 0.5], pv_gamma=[0.43, 0.3], dg_power=[300.0, 200.0], n_2=True,
                   dg_rating=300.0)
    dg, pmax, props, pvar, gamma = der_mix_properties(c)
    assert dg == 200.0 and gamma == 0.43
    np.testing.assert_array_equal(pmax, g1 + g2)
    np.testing.assert_array_equal(pvar, np.zeros(N) + g1 * 0.2 + g2 * 0.5)
    assert props["operation SOE min"] == 0.1 * 100.0 and props["operation SOE max"] == 0.95 * 100.0
    assert props["charge max"] == 20.0 and props["discharge max"] == 25.0 and props["rte"] == 0.9

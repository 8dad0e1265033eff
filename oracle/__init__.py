"""ORACLE -- test infrastructure only.

CPU restatement of the reference's per-window dispatch LP (DER-VET ``MicrogridScenario.optimize_problem_loop``
-> storagevet ``Scenario.set_up_optimization`` / ``solve_optimization``),
solved with HiGHS (scipy.optimize.linprog), plus a numpy restatement of the batched PDHG algorithm that the
HIP kernels implement (``pdlp_ref``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / CPU baseline.  The product path (``der-vet_amd/dervet_hip``) never
imports it.

Parity pinning: the restated LP + HiGHS reproduces the reference's golden per-window objective values
(``test/test_validation_report_sept1/Results/Usecase2/{es,es+pv+dg,es+pv}/step2/objective_values*.csv``,
25 windows) and the golden "Tariff Energy Price ($/kWh)" column; see ``tests/test_oracle_golden.py``.
"""

"""CPU oracle for the per-home HEMS MPC solve (dragg `mpc_calc.MPCCalc`).

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this package, and only as the
checker (or the timed CPU baseline) -- never as the thing measured or shipped.
The product path (`dragg_amd`) never imports it and fails loudly when its HIP
library is missing.

Contents
--------
`oracle.mpc`        numpy restatement of `dragg/mpc_calc.py` (problem build in the
                    reference's own variable / row order, solve, result extraction,
                    infeasibility fallback), solved with scipy HiGHS as the stand-in
                    for GLPK_MI (cvxpy/cvxopt/GLPK are absent from this image).
`oracle.community`  restatement of the aggregator's per-timestep loop
                    (`aggregator.py:711-778`: dispatch, collect_data sums).

Pinning: `tests/golden/*.json.gz` were produced by running the reference's own
code (tests/golden/make_golden.py); `tests/test_oracle_golden.py` checks this
oracle against them (matrices bit-for-bit, statuses, objectives, fallback
outputs, closed-loop collected data).
"""

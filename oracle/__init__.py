"""CPU oracle for the learner hot path — TEST INFRASTRUCTURE ONLY.

This package restates the reference HandyRL learner math on the CPU so the
HIP path can be checked against it.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker / the timed CPU baseline.  Nothing in
``handyrl_amd`` imports it: the product path runs on the HIP library or fails.

Pinning: every function here is checked against the golden vectors in
``tests/golden/`` that were produced by importing the reference itself
(``tests/golden/make_golden.py``); see ``tests/test_oracle_golden.py``.
"""

"""ORACLE -- test infrastructure only.

CPU restatements of the reference's VI-HMC log-posterior (and of hamiltorch's sampler) used as the
checker for the MI355X HIP path. Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import anything from here; the product (``vi-hmc_amd/vihmc``) never does.
The oracle is pinned by golden vectors generated from the reference itself (``tests/golden``).
"""

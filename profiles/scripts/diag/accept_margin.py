"""The accept margins (rho - log u) of test_inv_mass_fused_trajectory_vs_scalar_reference[bnn]'s scalar reference,
beside the engine runner's decisions with the native kinetic energy and with 0.5 * (p * p).sum(1): is a decision
that differs a borderline one (|rho - log u| within the Hamiltonian's fp32 rounding)?

    python profiles/scripts/diag/accept_margin.py
"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from goldens import bnn_case  # noqa: E402
from oracle import hamiltorch_ref as HR  # noqa: E402
from oracle.bnn_ref import TorchBNNRef, mlp_layout  # noqa: E402
from vihmc.engine import MLPEngine  # noqa: E402
from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner  # noqa: E402

dev = torch.device("cuda", 0)
c = bnn_case("bnn_vi_hmc")
g = c.g
sig = np.abs(np.asarray(g["mu"], np.float64)[c.idx]) * 0.1 + 0.01
spread = np.exp(np.random.default_rng(8).uniform(-np.log(2.0), np.log(2.0), sig.size))
inv_mass = torch.tensor(sig ** 2 / np.mean(sig ** 2) * spread, dtype=torch.float32)
th0 = torch.tensor(c.thetas[0])
S, L, eps, seeds = 12, 20, 5e-4, [40, 41]
fn = TorchBNNRef(mlp_layout(), c.data["x_train"], c.data["y_train"], g["mu"], c.idx,
                 prior_list=list(g["prior_var"]), loss=c.loss, tau_out=c.tau_out).log_prob
for native in (True, False):
    eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=2, device=dev)
    r = HMCRunner(EngineEvaluator(eng), th0[None].repeat(2, 1), S, L, eps, inv_mass=inv_mass,
                  rng=ChainRNG(2, th0.numel(), dev, seeds=seeds))
    r._native_ke = native
    for _ in range(S):
        r.step()
    acc = r.accepted.cpu()
    for ci, s in enumerate(seeds):
        gen = torch.Generator().manual_seed(s)
        _, st = HR.sample(fn, th0, S, L, eps, generator=gen, return_stats=True, inv_mass=inv_mass)
        diff = [i for i in range(S) if bool(acc[ci, i]) != st["accepts"][i]]
        margins = [round(a - b, 5) for a, b in zip(st["rhos"], st["logus"])]
        print(f"native_ke={native} chain {ci}: decisions differing from the reference at {diff}; reference "
              f"rho - log u = {margins}", flush=True)
    eng.close()

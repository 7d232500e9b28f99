"""Per-layer difference between the whole-network backward (bwd_chain = 1) and the per-layer launches (0) of one
single-chain full-parameter evaluation: python profiles/scripts/diag/chain_diff.py [--small]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

spec = DeepONetSpec()
small = "--small" in sys.argv
prob = deeponet_problem(seed=5, n=8, nt=11, nx=11, k=None) if small else deeponet_problem(seed=0, k=None)
D = spec.n_params
eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, np.arange(D), 0.0, 0.1,
                     "NLL", 1.0, max_chains=1, device="cuda:0")
th = torch.tensor(prob.mu, device="cuda:0")[None]
g = {}
for on in (0, 1):
    eng.option("bwd_chain", on)
    g[on] = eng.logp_grad(th)[1][0].double().cpu().numpy()
    print("bwd_chain", on, "->", eng.get_option("bwd_chain"))
for name, layers in (("branch", spec.branch), ("trunk", spec.trunk)):
    for j, L in enumerate(layers):
        for part, lo, hi in (("W", L.w_off, L.w_off + L.n_out * L.n_in), ("b", L.b_off, L.b_off + L.n_out)):
            a, b = g[0][lo:hi], g[1][lo:hi]
            d = np.abs(a - b)
            i = int(d.argmax())
            print(f"{name} {j} {part}: max|d| {d.max():.3e} rel {d.max() / max(np.abs(a).max(), 1e-30):.3e} "
                  f"ndiff {(d > 0).sum()} / {d.size} at {i} ({i // max(L.n_in, 1)}, {i % max(L.n_in, 1)}) "
                  f"ref {a[i]:.6e} got {b[i]:.6e}")
print("b0", g[0][0], g[1][0])

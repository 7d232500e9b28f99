"""Dump log p and its gradient of full-parameter Burgers evaluations (1 and 16 chains, seeded perturbations) from
the library VIHMC_LIB points at, for a bitwise comparison between two builds:

    VIHMC_LIB=a.so python profiles/scripts/diag/dump_eval.py out_a.npz
    VIHMC_LIB=b.so python profiles/scripts/diag/dump_eval.py out_b.npz
    python profiles/scripts/diag/dump_eval.py --compare out_a.npz out_b.npz
"""
import os
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = 0
    for k in a.files:
        d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64))
        n = int((a[k] != b[k]).sum())
        bad += n
        print(f"{k}: {n} of {a[k].size} elements differ, max |d| {d.max():.3e}")
    print("BITWISE EQUAL" if bad == 0 else "DIFFERENT")
    sys.exit(0 if bad == 0 else 1)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))
import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

spec = DeepONetSpec()
prob = deeponet_problem(seed=0, k=None)
out = {}
for C in (1, 16):
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu,
                         np.arange(spec.n_params), 0.0, 0.1, "NLL", 1.0, max_chains=C, device="cuda:0")
    gen = torch.Generator().manual_seed(C)
    th = torch.tensor(prob.mu)[None].repeat(C, 1)
    th += 1e-3 * torch.randn(th.shape, generator=gen, dtype=th.dtype)
    lp, g = eng.logp_grad(th.to("cuda:0"))
    out[f"logp_c{C}"] = lp.cpu().numpy()
    out[f"grad_c{C}"] = g.cpu().numpy()
    eng.close()
np.savez(sys.argv[1], **out)
print("wrote", sys.argv[1])

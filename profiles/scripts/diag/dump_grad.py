"""Dump gradient-only (Gram-form) evaluations of the Burgers problem at 16 distinct chains from the library VIHMC_LIB
points at, for a bitwise comparison between two builds (dump_eval.py covers the log-prob evaluations):

    VIHMC_LIB=a.so python profiles/scripts/diag/dump_grad.py out_a.npz
    python profiles/scripts/diag/dump_eval.py --compare out_a.npz out_b.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))
import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

spec = DeepONetSpec()
prob = deeponet_problem(seed=0, k=None)
out = {}
for C in (4, 16):
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu,
                         np.arange(spec.n_params), 0.0, 0.1, "NLL", 1.0, max_chains=C, device="cuda:0")
    gen = torch.Generator().manual_seed(C)
    th = torch.tensor(prob.mu)[None].repeat(C, 1)
    th += 1e-3 * torch.randn(th.shape, generator=gen, dtype=th.dtype)
    g = eng.grad(th.to("cuda:0"))
    assert eng.get_option("gram") & 2
    out[f"grad_c{C}"] = g.cpu().numpy()
    eng.close()
np.savez(sys.argv[1], **out)
print("wrote", sys.argv[1])

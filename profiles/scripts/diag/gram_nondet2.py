"""Which gradient evaluations of one plan differ, and after what? Sequences of grad / logp_grad calls on one plan at
the 64-function teacher shape (the guard test's) with distinct chains; prints, per option set, the calls whose
gradient differs from the first grad call (max |diff| per parameter segment) -- a stale-state dependency shows as
"the first call differs from the rest" or "a call after logp_grad differs"."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

dev = torch.device("cuda", 0)
spec = DeepONetSpec()


def segs(idx):
    lay = spec.branch + spec.trunk
    names = ["b0"] + [f"branch{i}" for i in range(len(spec.branch))] + [f"trunk{i}" for i in range(len(spec.trunk))]
    bounds = [0, 1] + [l.b_off + l.n_out for l in lay]
    return {nm: np.nonzero((idx >= bounds[k]) & (idx < bounds[k + 1]))[0] for k, nm in enumerate(names)}


def summary(d, sg, C):
    out = {}
    for c in range(C):
        for nm, ii in sg.items():
            m = float(d[c, ii].max()) if ii.size else 0.0
            if m > 0:
                out[f"c{c}:{nm}"] = m
    return out or "same"


p = deeponet_problem(seed=5, n=64, nt=21, nx=21, noise=1e-6, mu_noise=0.0)
sg = segs(p.grad_ind)
t = p.teacher[p.grad_ind].astype(np.float32)
rng = np.random.default_rng(4)
pert = [(t + 0.05 * rng.standard_normal(t.size)).astype(np.float32) for _ in range(2)]
th = torch.tensor(np.stack([t, t] + pert), device=dev)
C = 4
seqs = {"grad x5": "ggggg", "lg,g,g,lg,g,g": "lgglgg", "g,lg,g,lg,g": "glglg"}
for opts in ({}, {"bwd_chain": 0}, {"gram": 0}, {"gram": 0, "bwd_chain": 0}, {"bwd_bf16x6": 0},
             {"gram": 0, "bwd_bf16x6": 0}, {"contract_bf16x6": 0}):
    for sname, seq in seqs.items():
        eng = DeepONetEngine(spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, 0.0, 0.1, "NLL",
                             1.0, max_chains=C, device=dev)
        eng.option("gram_guard", 0)
        for k, v in opts.items():
            eng.option(k, v)
        res = []
        for ch in seq:
            if ch == "g":
                res.append(("g", eng.grad(th).cpu().numpy()))
            else:
                res.append(("lg", eng.logp_grad(th)[1].cpu().numpy()))
        g0 = next(r for kind, r in res if kind == "g")
        lg0 = next((r for kind, r in res if kind == "lg"), None)
        line = []
        for i, (kind, r) in enumerate(res):
            ref = g0 if kind == "g" else lg0
            line.append(f"{i}:{kind}={summary(np.abs(r - ref), sg, C)}")
        print(f"{opts} [{sname}] bwd_chain={eng.get_option('bwd_chain')} gram={eng.get_option('gram')}: "
              + " | ".join(line), flush=True)
        eng.close()

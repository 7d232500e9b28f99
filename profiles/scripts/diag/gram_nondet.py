"""Is the Gram-form gradient bitwise repeatable? Repeated vihmc_grad calls on one plan, per chain count and problem;
reports the largest difference per parameter segment (output bias, branch layers, trunk layers) and the split sizes."""
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
    out = {}
    for k, nm in enumerate(names):
        out[nm] = np.nonzero((idx >= bounds[k]) & (idx < bounds[k + 1]))[0]
    return out


for name, kw in [("teacher64", dict(seed=5, n=64, nt=21, nx=21, noise=1e-6, mu_noise=0.0)),
                 ("noisy64", dict(seed=5, n=64, nt=21, nx=21, noise=1e-2, mu_noise=0.01)),
                 ("burgers", dict(seed=0))]:
    p = deeponet_problem(**kw)
    sg = segs(p.grad_ind)
    rng = np.random.default_rng(4)
    base = p.mu[p.grad_ind]
    for C in (2, 4):
        for opts in ({}, {"bwd_chain": 0}, {"gram": 0}):
            eng = DeepONetEngine(spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, 0.0, 0.1, "NLL",
                                 1.0, max_chains=C, device=dev)
            eng.option("gram_min_chains", 1)
            eng.option("gram_guard", 0)
            for k, v in opts.items():
                eng.option(k, v)
            # distinct chains (a cross-chain race is invisible with identical chains)
            th = torch.tensor(np.stack([base + 0.02 * c * rng.standard_normal(base.size) for c in range(C)]).astype(np.float32),
                              device=dev)
            gs = [eng.grad(th).cpu().numpy() for _ in range(5)]
            bad = {}
            for k in range(1, 5):
                d = np.abs(gs[k] - gs[0])
                for c in range(C):
                    for nm, ii in sg.items():
                        m = float(d[c, ii].max()) if ii.size else 0.0
                        if m > 0:
                            bad[f"c{c}:{nm}"] = max(bad.get(f"c{c}:{nm}", 0.0), m)
            print(f"{name} C={C} {opts} bwd_chain ran={eng.get_option('bwd_chain')} gram ran={eng.get_option('gram')}: "
                  f"repeat diffs {bad or 'none'}", flush=True)
            eng.close()

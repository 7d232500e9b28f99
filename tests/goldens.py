"""Loading of the reference-generated golden fixtures (tests/golden/*.npz, see make_golden.py)."""
from __future__ import annotations

import hashlib
import os
from types import SimpleNamespace

import numpy as np

from vihmc.data import deeponet_problem
from vihmc.layout import DeepONetSpec, MLPSpec

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

BNN_CASES = ["bnn_vi_hmc", "bnn_hmc_regression", "bnn_load_prior", "bnn_tensor_prior"]
DEEPONET_CASES = ["deeponet_small", "deeponet_small_loadprior", "deeponet_odd_full", "deeponet_refshape"]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def spec_of(g) -> DeepONetSpec:
    wb, wt, ib, it, db, dt, out = (int(v) for v in g["spec"])
    return DeepONetSpec(width_branch=wb, width_trunk=wt, in_branch=ib, in_trunk=it, depth_branch=db, depth_trunk=dt,
                        output_neurons=out)


def refshape_theta1(th0):
    return (th0 + 0.01 * np.random.default_rng(7).standard_normal(th0.size)).astype(np.float32)


def deeponet_case(name: str):
    """Inputs + expected outputs of a DeepONet golden case (regenerating seeded inputs when the
    fixture stores only their checksums)."""
    g = load(name)
    spec = spec_of(g)
    if "branch_in" in g:
        prob = SimpleNamespace(branch_in=g["branch_in"], trunk_in=g["trunk_in"], y=g["y"], mu=g["mu"],
                               sigma=g["sigma"], grad_ind=g["grad_ind"])
        thetas = [g["theta0"], g["theta1"]]
    else:
        p = deeponet_problem(seed=int(g["seed"]), n=int(g["n"]), nt=int(g["nt"]), nx=int(g["nx"]), spec=spec,
                             k=int(g["k"]))
        for key, arr in (("sha_branch", p.branch_in), ("sha_trunk", p.trunk_in), ("sha_y", p.y), ("sha_mu", p.mu),
                         ("sha_idx", p.grad_ind)):
            assert sha(arr) == str(g[key]), f"{name}: regenerated input {key} drifted from the golden fixture"
        prob = p
        th0 = p.mu[p.grad_ind]
        thetas = [th0] + ([refshape_theta1(th0)] if "logp1" in g else [])
        for t, th in enumerate(thetas):
            assert sha(th) == str(g[f"theta{t}_sha"])
    prior_mu, prior_sd = (0.0, float(np.sqrt(g["prior_var"])))
    if bool(g["load_prior"]):
        prior_mu, prior_sd = prob.mu[prob.grad_ind], prob.sigma[prob.grad_ind]
    return SimpleNamespace(g=g, spec=spec, prob=prob, thetas=thetas, prior_mu=prior_mu, prior_sd=prior_sd,
                           loss=str(g["loss"]), tau_out=float(g["tau_out"]), full=len(prob.grad_ind) == spec.n_params)


def split_theta1(th0, seed=8):
    return (th0 + 0.01 * np.random.default_rng(seed).standard_normal(th0.size)).astype(np.float32)


def split_burgers_case():
    """Config 4 at the reference shape (make_golden.deeponet_split_burgers_cases): the full-parameter
    Burgers problem split into two contiguous shards of N/2 functions, inputs regenerated from the seed
    and checked against the fixture's SHA-256s."""
    g = load("deeponet_split_burgers")
    spec = spec_of(g)
    p = deeponet_problem(seed=int(g["seed"]), n=int(g["n"]), nt=int(g["nt"]), nx=int(g["nx"]), spec=spec, k=None)
    for key, arr in (("sha_branch", p.branch_in), ("sha_trunk", p.trunk_in), ("sha_y", p.y), ("sha_mu", p.mu),
                     ("sha_sigma", p.sigma)):
        assert sha(arr) == str(g[key]), f"deeponet_split_burgers: regenerated input {key} drifted"
    th0 = p.mu.copy()
    thetas = [th0, split_theta1(th0, int(g["theta1_seed"]))]
    for t, th in enumerate(thetas):
        assert sha(th) == str(g[f"theta{t}_sha"])
    half = p.N // 2
    shards = [(p.branch_in[m * half:(m + 1) * half], p.trunk_in, p.y[m * half:(m + 1) * half]) for m in range(2)]
    return SimpleNamespace(g=g, spec=spec, prob=p, thetas=thetas, shards=shards, loss=str(g["loss"]),
                           tau_out=float(g["tau_out"]), prior_sd=float(np.sqrt(g["prior_var"])))


def bnn_case(name: str):
    g = load(name)
    data = load("bnn_data")
    spec = MLPSpec()
    idx = g["grad_ind"]
    K = idx.size
    if bool(g["load_prior"]):
        pm, ps = g["mu"][idx], g["sd"][idx]
    else:
        from vihmc.engine import prior_per_tensor
        pm, ps = 0.0, prior_per_tensor(spec.tensor_sizes, K, np.sqrt(g["prior_var"]))
    return SimpleNamespace(g=g, spec=spec, data=data, idx=idx, prior_mu=pm, prior_sd=ps, loss=str(g["loss"]),
                           tau_out=float(g["tau_out"]), thetas=[g["theta0"], g["theta1"]])

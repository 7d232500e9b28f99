"""Gram-form gradient-only contraction (vihmc_grad; vihmc_gram.hip) vs the reference goldens, the fp64 oracle and
the residual-form path, through the C-ABI.

The Gram form computes dZ_b = gscale (Zb^ Zt^T Zt^ - y Zt^) and dZ_t = gscale (Zt^ Zb^T Zb^ - y^T Zb^) (augmented
outputs Zb^ = [Z_b | 1], Zt^ = [Z_t | b0]) instead of forming G = gscale (S + b0 - y): algebraically the reference's
autograd backward of my_make_func.py:79-82 + the Gaussian NLL (main_VI_HMC_burgers.py:157-163); its rounding
differs from the residual form by the cancellation between Zb^ Gt and y Zt^, so it has its own recorded bounds.
"""
import numpy as np
import pytest
import torch

import parity
from goldens import deeponet_case
from oracle.deeponet_ref import deeponet_layout, np_logp_grad

pytestmark = pytest.mark.gpu


def engine_for(c, max_chains, device, min_chains=2):
    from vihmc.engine import DeepONetEngine, trunk_features
    p = c.prob
    eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                         c.prior_sd, c.loss, c.tau_out, max_chains=max_chains, device=device)
    eng.option("gram_min_chains", min_chains)       # the tests run the Gram form from 2 chains (default 4)
    return eng


def rel_norm(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.parametrize("C", [2, 3, 16])
def test_gram_grad_burgers_matches_golden(C, cuda_device):
    """Full Burgers shape (N = 1000, P = 10,201, W = 100): every chain's Gram-form gradient against the reference
    closure's golden (4,096-entry subsample + the norm of the whole gradient) and against the residual form."""
    c = deeponet_case("deeponet_burgers")
    eng = engine_for(c, C, cuda_device)
    n = len(c.thetas)
    th = torch.tensor(np.stack([c.thetas[i % n] for i in range(C)]), device=cuda_device)
    g = eng.grad(th).cpu().numpy()
    assert eng.get_option("gram") & 2, "the Gram form did not run"
    _, gr = eng.logp_grad(th)
    gr = gr.cpu().numpy()
    assert not eng.get_option("gram") & 2
    sub = c.g["grad_subsample"]
    for i in range(C):
        t = i % n
        gs = c.g[f"grad{t}_sub"]
        note = f"C={C} chain {i}"
        parity.check("grad_elem", np.abs(g[i][sub] - gs).max() / np.abs(gs).max(), note)
        nrm = float(c.g[f"grad{t}_norm"])
        parity.check("grad_norm_rel", abs(np.linalg.norm(g[i]) - nrm) / nrm, note)
        parity.check("grad_relnorm", rel_norm(g[i], gr[i]), note + " vs residual form")


def test_gram_grad_refshape_vs_fp64_oracle(cuda_device):
    """Reference shapes (W = 100, 8 x 121 points): full gradients against the fp64 oracle, 4 chains."""
    c = deeponet_case("deeponet_refshape")
    p = c.prob
    C = 4
    rng = np.random.default_rng(5)
    thetas = [np.asarray(c.thetas[i % len(c.thetas)], np.float32) +
              (0.02 * rng.standard_normal(len(c.thetas[0]))).astype(np.float32) * (i > 1) for i in range(C)]
    eng = engine_for(c, C, cuda_device)
    g = eng.grad(torch.tensor(np.stack(thetas), device=cuda_device)).cpu().numpy()
    assert eng.get_option("gram") & 2
    s = c.spec
    lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk,
                          s.out)
    for i, th in enumerate(thetas):
        _, rg, _ = np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, th, c.prior_mu, c.prior_sd,
                                c.loss, c.tau_out)
        parity.check("grad_relnorm", rel_norm(g[i], rg), f"chain {i}")
        parity.check("grad_elem", np.abs(g[i] - rg).max() / np.abs(rg).max(), f"chain {i}")


def test_gram_option_off_is_the_residual_form(cuda_device):
    """gram = 0 (or fewer chains than gram_min_chains): vihmc_grad is bitwise the gradient of vihmc_logp_grad; the
    default threshold is 4 chains."""
    c = deeponet_case("deeponet_refshape")
    eng = engine_for(c, 2, cuda_device)
    th = torch.tensor(np.stack(c.thetas[:2]), device=cuda_device)
    _, gr = eng.logp_grad(th)
    assert eng.get_option("gram_min_chains") == 2
    eng.option("gram", 0)
    g = eng.grad(th)
    assert not eng.get_option("gram") & 2
    assert torch.equal(g, gr)
    eng.option("gram", 1)
    g1 = eng.grad(th[:1])            # C = 1 < gram_min_chains (2 here)
    assert not eng.get_option("gram") & 2
    assert torch.equal(g1, gr[:1])


def test_gram_after_set_data_and_trunk_rows(cuda_device):
    """The pre-split data images follow vihmc_plan_set_data and vihmc_plan_set_trunk_rows (cfg.sample_data)."""
    c = deeponet_case("deeponet_refshape")
    p = c.prob
    eng = engine_for(c, 2, cuda_device)
    th = torch.tensor(np.stack(c.thetas[:2]), device=cuda_device)
    y2 = torch.tensor(p.y[::-1].copy(), device=cuda_device)
    eng.set_data(torch.tensor(p.branch_in[::-1].copy(), device=cuda_device), y2)
    g = eng.grad(th).cpu().numpy()
    _, gr = eng.logp_grad(th)
    parity.check("grad_relnorm", max(rel_norm(g[i], gr[i].cpu().numpy()) for i in range(2)), "set_data")
    from vihmc.engine import trunk_features
    feat = torch.tensor(trunk_features(p.trunk_in), device=cuda_device)
    eng.set_sample_grid(feat, y2)
    ind = np.random.default_rng(3).permutation(p.y.shape[1]).astype(np.int32)
    eng.set_trunk_rows(ind)
    g = eng.grad(th).cpu().numpy()
    _, gr = eng.logp_grad(th)
    parity.check("grad_relnorm", max(rel_norm(g[i], gr[i].cpu().numpy()) for i in range(2)), "set_trunk_rows")


def test_gram_deterministic(cuda_device):
    """Fixed-order reductions only (split-K slabs, Gram slabs, d ll / d b0 slots): repeated calls are bitwise equal."""
    c = deeponet_case("deeponet_burgers")
    eng = engine_for(c, 4, cuda_device)
    th = torch.tensor(np.stack([c.thetas[i % len(c.thetas)] for i in range(4)]), device=cuda_device)
    a = eng.grad(th).clone()
    for _ in range(3):
        assert torch.equal(eng.grad(th), a)


@pytest.mark.parametrize("form", ["gram", "residual"])
def test_full_shape_grad_vs_fp64_oracle(form, cuda_device):
    """Full Burgers shape, the golden theta and a perturbed copy: the gradient of each contraction form against the fp64 oracle (the
    reference's own fp32 closure is within ~1e-7 of it: its goldens' grad subsample). Records how much precision the
    Gram form's cancellation (Zb^ Gt vs y Zt^, sums over P = 10,201 points) costs next to the residual form."""
    c = deeponet_case("deeponet_burgers")
    p = c.prob
    s = c.spec
    eng = engine_for(c, 2, cuda_device)
    th0 = np.asarray(c.thetas[0], np.float32)
    thetas = [th0, (th0 + 0.01 * np.random.default_rng(11).standard_normal(th0.size)).astype(np.float32)]
    th = torch.tensor(np.stack(thetas), device=cuda_device)
    g = (eng.grad(th) if form == "gram" else eng.logp_grad(th)[1]).cpu().numpy()
    assert bool(eng.get_option("gram") & 2) == (form == "gram")
    lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk,
                          s.out)
    for i in range(2):
        _, rg, _ = np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, thetas[i], c.prior_mu,
                                c.prior_sd, c.loss, c.tau_out)
        parity.check("grad_relnorm", rel_norm(g[i], rg), f"{form} theta{i}")
        parity.check("grad_elem", np.abs(g[i] - rg).max() / np.abs(rg).max(), f"{form} theta{i}")


@pytest.mark.parametrize("loss,tau", [("regression", 2.5), ("NLL", 0.3)])
def test_gram_loss_forms_vs_fp64_oracle(loss, tau, cuda_device):
    """Both Gaussian likelihood forms (gscale = -1/tau for 'NLL', -tau for 'regression') and a non-unit tau through
    the Gram form, against the fp64 oracle at the reference shapes (4 chains)."""
    from vihmc.engine import DeepONetEngine, trunk_features
    c = deeponet_case("deeponet_refshape")
    p, s = c.prob, c.spec
    C = 4
    rng = np.random.default_rng(9)
    thetas = [np.asarray(c.thetas[i % len(c.thetas)], np.float32) +
              (0.02 * rng.standard_normal(len(c.thetas[0]))).astype(np.float32) * (i > 1) for i in range(C)]
    eng = DeepONetEngine(s, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd,
                         loss, tau, max_chains=C, device=cuda_device)
    g = eng.grad(torch.tensor(np.stack(thetas), device=cuda_device)).cpu().numpy()
    assert eng.get_option("gram") & 2
    lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk,
                          s.out)
    for i, th in enumerate(thetas):
        _, rg, _ = np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, th, c.prior_mu, c.prior_sd,
                                loss, tau)
        parity.check("grad_relnorm", rel_norm(g[i], rg), f"{loss} tau={tau} chain {i}")

"""CPU checks of the Bayesian DeepONet VI training surface (vihmc/vi.py) against the reference's own
train_model / validate_model / metrics.mse outputs (tests/golden/vi_deeponet_*.npz): initialisation draws,
weight-noise draw order (through the float64 oracle oracle/vi_ref.py), KL, ELBO / MSE values, and the host
logic that maps each item's permuted trunk points back to the grid order."""
import numpy as np
import pytest
import torch

from oracle.vi_ref import elbo_step, eval_loss
from vi_cases import NOISE_CASE, VI_CASES, make_model, rel_norm, vi_case


@pytest.mark.parametrize("name", VI_CASES)
def test_init_matches_reference(name):
    c = vi_case(name)
    m = make_model(c)
    assert np.array_equal(m.mu_flat().detach().numpy(), c.g["mu0"])
    assert np.array_equal(m.rho_flat().detach().numpy(), c.g["rho0"])


@pytest.mark.parametrize("name", VI_CASES)
def test_oracle_step_with_our_draws_matches_reference(name):
    """Our draw order + the float64 oracle ELBO reproduce the reference's loss and mu / rho gradients."""
    c = vi_case(name)
    m = make_model(c)
    torch.manual_seed(c.seed + 1000)
    eps = [m.draw_eps().numpy() for _ in range(c.num_ens)]
    from vihmc.vi import get_beta
    beta = get_beta(0, 1, c.beta, None, None)
    loss, gm, gr = elbo_step(c.layout, c.g["mu0"], c.g["rho0"], eps, c.g["branch_in"], c.g["trunk_grid"],
                             c.g["y_grid"], beta, c.train_size, act=c.act)
    assert loss == pytest.approx(float(c.g["loss_train"]), rel=2e-6)
    assert rel_norm(gm, c.g["grad_mu"]) < 1e-5
    assert rel_norm(gr, c.g["grad_rho"]) < 1e-5


@pytest.mark.parametrize("name", VI_CASES)
def test_eval_loss_mse_and_kl(name):
    """After the recorded step the reference validated with the unchanged parameters (the recorder did
    not update them): eval-mode loss, MSE and KL."""
    c = vi_case(name)
    m = make_model(c)
    from vihmc.vi import get_beta
    beta = get_beta(0, 1, c.beta, None, None)
    lv, mv = eval_loss(c.layout, c.g["mu0"], c.g["rho0"], c.g["branch_in"], c.g["trunk_grid"], c.g["y_grid"], beta,
                       c.train_size, act=c.act)
    assert lv == pytest.approx(float(c.g["loss_val"]), rel=2e-6)
    assert mv == pytest.approx(float(c.g["mse_val"]), rel=1e-5)
    assert float(m.kl()) == pytest.approx(float(c.g["kl0"]), rel=1e-6)


def test_canonical_undoes_item_permutations():
    from vihmc.layout import DeepONetSpec
    from vihmc.vi import BatchEngines
    c = vi_case("vi_deeponet_tanh")
    be = BatchEngines(DeepONetSpec(12, 12, 7, 5, 3, 3, "tanh", 12), c.g["trunk_grid"], 1.0, 2, "cuda")
    y, count = be.canonical(c.batch[1], c.batch[2])
    assert torch.equal(y, torch.from_numpy(c.g["y_grid"]))
    assert count == y.numel()
    bad = c.batch[1].clone()
    bad[0, 0] = bad[0, 1]                      # a repeated point: not distinct grid points
    with pytest.raises(ValueError):
        be.canonical(bad, c.batch[2])


def test_canonical_per_item_subsets():
    """p < P (utils.py:39-41 draws p of the P trunk points per item): each item's targets land on its own grid
    points, the points it did not draw hold NaN (the engine's masked plans skip them), count = B p."""
    from vihmc.layout import DeepONetSpec
    from vihmc.vi import BatchEngines
    c = vi_case("vi_deeponet_tanh")
    grid = c.g["trunk_grid"].reshape(-1, 2)
    P = grid.shape[0]
    be = BatchEngines(DeepONetSpec(12, 12, 7, 5, 3, 3, "tanh", 12), grid, 1.0, 2, "cuda")
    rng = np.random.default_rng(3)
    B, p = 4, P // 3
    ind = np.stack([rng.choice(P, p, replace=False) for _ in range(B)])
    yfull = rng.standard_normal((B, P)).astype(np.float32)
    xt = torch.from_numpy(grid[ind])
    yt = torch.from_numpy(np.take_along_axis(yfull, ind, 1))
    y, count = be.canonical(xt, yt)
    assert count == B * p
    mask = np.zeros((B, P), bool)
    np.put_along_axis(mask, ind, True, 1)
    yn = y.numpy()
    assert np.array_equal(np.isnan(yn), ~mask)
    assert np.array_equal(yn[mask], yfull[mask])


def test_elbo_module_matches_formula():
    from vihmc.vi import ELBO, calculate_kl
    torch.manual_seed(0)
    pred, y = torch.randn(3, 7), torch.randn(3, 7)
    kl = calculate_kl(0, 0.1, torch.randn(5), torch.rand(5) + 0.05)
    v = ELBO()(pred, y, kl, 0.5, 100, torch.tensor(2.0))
    ref = 100 * torch.mean(0.5 * (np.log(2.0) + (pred - y) ** 2 / 2.0)) + 0.5 * kl
    assert float(v) == pytest.approx(float(ref), rel=1e-6)


def test_learn_noise_case_matches_reference():
    """learn_noise, noise_type 0 (main_VI_deeponet.py:154-156, metrics.py:21-25): the log-variance draw after the
    model, and the float64 oracle's loss and mu / rho / log-variance gradients with our weight-noise draws, against
    the reference's own train_model / validate_model (tests/golden/vi_deeponet_noise.npz)."""
    from vihmc.vi import get_beta
    c = vi_case(NOISE_CASE)
    assert bool(c.g["learn_noise"])
    m = make_model(c)
    noise0 = torch.randn((1))
    assert np.array_equal(noise0.numpy(), c.g["noise0"])
    torch.manual_seed(c.seed + 1000)
    eps = [m.draw_eps().numpy() for _ in range(c.num_ens)]
    beta = get_beta(0, 1, c.beta, None, None)
    lv = float(c.g["noise0"][0])
    loss, gm, gr, gl = elbo_step(c.layout, c.g["mu0"], c.g["rho0"], eps, c.g["branch_in"], c.g["trunk_grid"],
                                 c.g["y_grid"], beta, c.train_size, act=c.act, log_var=lv)
    assert loss == pytest.approx(float(c.g["loss_train"]), rel=2e-6)
    assert rel_norm(gm, c.g["grad_mu"]) < 1e-5
    assert rel_norm(gr, c.g["grad_rho"]) < 1e-5
    assert gl == pytest.approx(float(c.g["grad_noise"][0]), rel=1e-4)
    lval, _ = eval_loss(c.layout, c.g["mu0"], c.g["rho0"], c.g["branch_in"], c.g["trunk_grid"], c.g["y_grid"], beta,
                        c.train_size, act=c.act, log_var=lv)
    assert lval == pytest.approx(float(c.g["loss_val"]), rel=2e-6)


def test_elbo_module_learn_noise_and_unsupported_head():
    from vihmc.vi import ELBO, Bayesian_DeepONet, _check_loss, calculate_kl
    torch.manual_seed(1)
    pred, y = torch.randn(3, 7), torch.randn(3, 7)
    kl = calculate_kl(0, 0.1, torch.randn(5), torch.rand(5) + 0.05)
    lv = torch.tensor([0.3], requires_grad=True)
    v = ELBO(True, 0)(pred, y, kl, 0.5, 100, lv)
    ref = 100 * torch.mean(0.5 * (0.3 + (pred - y) ** 2 / np.exp(0.3))) + 0.5 * kl
    assert float(v) == pytest.approx(float(ref), rel=1e-6)
    v.backward()
    dref = 100 * float(torch.mean(0.5 * (1 - (pred - y) ** 2 / np.exp(0.3))))
    assert float(lv.grad) == pytest.approx(dref, rel=1e-5)
    with pytest.raises(NotImplementedError):
        _check_loss(ELBO(True, 1))
    with pytest.raises(NotImplementedError):
        Bayesian_DeepONet({"prior_mu": 0, "prior_sigma": 0.1, "posterior_mu_initial": (0, 0.1),
                           "posterior_rho_initial": (-5, 0.1)}, 8, 8, 3, 5, 3, 3, 10, "tanh", 1, 2)

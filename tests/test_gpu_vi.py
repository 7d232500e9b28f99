"""Bayesian DeepONet VI training on the GPU (vihmc/vi.py: the NLL part of every ELBO through the HIP engine)
against the reference's own train_model / validate_model / metrics.mse (tests/golden/vi_deeponet_*.npz), and
at the Burgers shapes (width 100, depth 9, 101 x 101 grid) against the float64 oracle (oracle/vi_ref.py)."""
import time

import numpy as np
import pytest
import torch

from oracle.vi_ref import elbo_step
from vi_cases import NOISE_CASE, VI_CASES, GradRecorder, make_model, rel_norm, vi_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", VI_CASES)
def test_train_validate_mse_match_reference(name, cuda_device):
    from vihmc.vi import ELBO, BatchEngines, mse, train_model, validate_model
    c = vi_case(name)
    m = make_model(c).to(cuda_device)
    eng = BatchEngines(m.spec, c.g["trunk_grid"], 1.0, c.num_ens, cuda_device)
    try:
        rec = GradRecorder(m)
        torch.manual_seed(c.seed + 1000)
        lt = train_model([c.batch], m, ELBO(), rec, c.train_size, 1, c.num_ens, c.beta, engines=eng)
        assert lt == pytest.approx(float(c.g["loss_train"]), rel=2e-5)
        assert rel_norm(rec.grads[0].cpu().numpy(), c.g["grad_mu"]) < 2e-4
        assert rel_norm(rec.grads[1].cpu().numpy(), c.g["grad_rho"]) < 2e-4
        lv = validate_model([c.batch], m, ELBO(), c.train_size, c.beta, 1, engines=eng)
        assert lv == pytest.approx(float(c.g["loss_val"]), rel=2e-5)
        assert mse([c.batch], m, engines=eng) == pytest.approx(float(c.g["mse_val"]), rel=1e-4)
    finally:
        eng.close()


def test_learn_noise_train_validate_match_reference(cuda_device):
    """learn_noise (noise_type 0): the trainable log-variance through train_model / validate_model -- loss and the
    mu / rho / log-variance gradients against the reference's own step (tests/golden/vi_deeponet_noise.npz)."""
    from vihmc.vi import ELBO, BatchEngines, train_model, validate_model
    c = vi_case(NOISE_CASE)
    m = make_model(c)
    noise = torch.nn.Parameter(torch.randn((1)).to(cuda_device))
    assert np.array_equal(noise.detach().cpu().numpy(), c.g["noise0"])
    m = m.to(cuda_device)
    eng = BatchEngines(m.spec, c.g["trunk_grid"], 1.0, c.num_ens, cuda_device)
    try:
        rec = GradRecorder(m)
        torch.manual_seed(c.seed + 1000)
        loss = ELBO(True, 0)
        lt = train_model([c.batch], m, loss, rec, c.train_size, 1, c.num_ens, c.beta, noise_param=noise, engines=eng)
        assert lt == pytest.approx(float(c.g["loss_train"]), rel=2e-5)
        assert rel_norm(rec.grads[0].cpu().numpy(), c.g["grad_mu"]) < 2e-4
        assert rel_norm(rec.grads[1].cpu().numpy(), c.g["grad_rho"]) < 2e-4
        assert float(noise.grad) == pytest.approx(float(c.g["grad_noise"][0]), rel=2e-3)
        lv = validate_model([c.batch], m, loss, c.train_size, c.beta, 1, noise_param=noise, engines=eng)
        assert lv == pytest.approx(float(c.g["loss_val"]), rel=2e-5)
        with pytest.raises(ValueError):             # learn_noise needs variance-1 plans
            bad = BatchEngines(m.spec, c.g["trunk_grid"], 2.0, c.num_ens, cuda_device)
            try:
                validate_model([c.batch], m, loss, c.train_size, c.beta, 1, noise_param=noise, engines=bad)
            finally:
                bad.close()
    finally:
        eng.close()


def test_burgers_shape_step_matches_oracle(cuda_device):
    """Width 100, depth 9, the 101 x 101 grid, 6 functions with permuted points, 2 weight draws: one training
    step's loss and gradients against the float64 oracle; plus the data swap between two batches."""
    from oracle.deeponet_ref import deeponet_layout
    from vihmc.data import deeponet_problem
    from vihmc.vi import ELBO, BatchEngines, Bayesian_DeepONet, train_model
    prob = deeponet_problem(seed=3, n=12)
    grid = prob.trunk_in[0]
    P = grid.shape[0]
    priors = {"prior_mu": 0, "prior_sigma": 0.1, "posterior_mu_initial": (0, 0.1), "posterior_rho_initial": (-5, 0.1)}
    torch.manual_seed(7)
    m = Bayesian_DeepONet(priors, 100, 100, 101, 5, 9, 9, 100, "tanh", 0, 0, impose_bc=True)
    mu0, rho0 = m.mu_flat().detach().numpy().copy(), m.rho_flat().detach().numpy().copy()
    m = m.to(cuda_device)
    rng = np.random.default_rng(5)
    batches = []
    for b0 in (0, 6):
        perms = np.stack([rng.permutation(P) for _ in range(6)])
        batches.append((torch.from_numpy(prob.branch_in[b0:b0 + 6]),
                        torch.from_numpy(np.stack([grid[p] for p in perms])),
                        torch.from_numpy(np.stack([prob.y[b0 + i, perms[i]] for i in range(6)]))))
    eng = BatchEngines(m.spec, grid, 1.0, 2, cuda_device)
    lay = deeponet_layout()
    try:
        for bi, batch in enumerate(batches):
            rec = GradRecorder(m)
            torch.manual_seed(100 + bi)
            eps = [m.draw_eps().numpy() for _ in range(2)]
            torch.manual_seed(100 + bi)
            lt = train_model([batch], m, ELBO(), rec, 1000 * P, 1, 2, 1.0, engines=eng)
            b0 = 6 * bi
            loss, gm, gr = elbo_step(lay, mu0, rho0, eps, prob.branch_in[b0:b0 + 6, 0], grid, prob.y[b0:b0 + 6], 1.0,
                                     1000 * P)
            assert lt == pytest.approx(loss, rel=2e-5)
            assert rel_norm(rec.grads[0].cpu().numpy(), gm) < 2e-4
            assert rel_norm(rec.grads[1].cpu().numpy(), gr) < 2e-4
    finally:
        eng.close()


def _subset_batch(branch_in, grid, y_grid, p, seed):
    """Items with their own p of the P grid points (utils.py:39-41: np.random.choice(P, p, replace=False) per
    item): the batch as the reference's loader yields it, and y_grid with NaN at each item's undrawn points."""
    rng = np.random.default_rng(seed)
    B, P = y_grid.shape
    ind = np.stack([rng.choice(P, p, replace=False) for _ in range(B)])
    batch = (torch.from_numpy(np.ascontiguousarray(branch_in)).view(B, 1, -1), torch.from_numpy(grid[ind]),
             torch.from_numpy(np.take_along_axis(y_grid, ind, 1)))
    y_nan = np.full_like(y_grid, np.nan)
    np.put_along_axis(y_nan, ind, np.take_along_axis(y_grid, ind, 1), 1)
    return batch, y_nan


@pytest.mark.parametrize("shape", ["small", "burgers"])
def test_per_item_trunk_subsets_match_oracle(shape, cuda_device):
    """p < P: every item carries its own random subset of the trunk grid. The engine runs the whole grid with the
    undrawn (item, point) pairs as NaN targets (plan option y_masked: residual 0 there; lik_count = B p), so one
    training step's loss and mu / rho gradients, the eval-mode loss and the MSE match the float64 oracle's mean over
    the drawn pairs. small = the golden case's width-12 network (fp32 contraction), burgers = width 100, 101 x 101
    grid (bf16x6 contraction). Parity unpinned against the reference itself: its golden batches carry p = P."""
    from oracle.deeponet_ref import deeponet_layout
    from oracle.vi_ref import eval_loss
    from vihmc.vi import ELBO, BatchEngines, Bayesian_DeepONet, mse, train_model, validate_model
    if shape == "small":
        c = vi_case("vi_deeponet_tanh")
        m = make_model(c)
        grid = c.g["trunk_grid"].reshape(-1, 2)
        y_grid, branch = c.g["y_grid"], c.g["branch_in"].reshape(c.B, -1)
        lay, act, size = c.layout, c.act, c.train_size
    else:
        from vihmc.data import deeponet_problem
        prob = deeponet_problem(seed=3, n=6)
        grid = prob.trunk_in[0]
        priors = {"prior_mu": 0, "prior_sigma": 0.1, "posterior_mu_initial": (0, 0.1),
                  "posterior_rho_initial": (-5, 0.1)}
        torch.manual_seed(7)
        m = Bayesian_DeepONet(priors, 100, 100, 101, 5, 9, 9, 100, "tanh", 0, 0, impose_bc=True)
        y_grid, branch = prob.y, prob.branch_in[:, 0]
        lay, act, size = deeponet_layout(), "tanh", 1000 * grid.shape[0]
    P = grid.shape[0]
    batch, y_nan = _subset_batch(branch, grid, y_grid, P // 3, 11)
    mu0, rho0 = m.mu_flat().detach().numpy().copy(), m.rho_flat().detach().numpy().copy()
    m = m.to(cuda_device)
    eng = BatchEngines(m.spec, grid, 1.0, 2, cuda_device)
    try:
        rec = GradRecorder(m)
        torch.manual_seed(31)
        eps = [m.draw_eps().numpy() for _ in range(2)]
        torch.manual_seed(31)
        lt = train_model([batch], m, ELBO(), rec, size, 1, 2, 1.0, engines=eng)
        e0 = eng.get(batch[0].shape[0])
        assert e0.get_option("y_masked") == 1 and e0.get_option("lik_count") == y_grid.shape[0] * (P // 3)
        assert not (e0.get_option("gram") & 2)
        loss, gm, gr = elbo_step(lay, mu0, rho0, eps, branch, grid, y_nan, 1.0, size, act=act)
        assert lt == pytest.approx(loss, rel=2e-5)
        assert rel_norm(rec.grads[0].cpu().numpy(), gm) < 2e-4
        assert rel_norm(rec.grads[1].cpu().numpy(), gr) < 2e-4
        lv_ref, mse_ref = eval_loss(lay, mu0, rho0, branch, grid, y_nan, 1.0, size, act=act)
        lv = validate_model([batch], m, ELBO(), size, 1.0, 1, engines=eng)
        assert lv == pytest.approx(lv_ref, rel=2e-5)
        assert mse([batch], m, engines=eng) == pytest.approx(mse_ref, rel=1e-4)
        # a whole-grid batch on the same plan clears the mask again
        full = (batch[0], torch.from_numpy(np.broadcast_to(grid, (y_grid.shape[0],) + grid.shape).copy()),
                torch.from_numpy(np.ascontiguousarray(y_grid, dtype=np.float32)))
        eng.load(full)
        assert e0.get_option("y_masked") == 0 and e0.get_option("lik_count") == y_grid.shape[0] * P
    finally:
        eng.close()


def test_burgers_training_step_timing(cuda_device):
    """main_VI_deeponet's configuration: batch 128 functions x 10,201 points, num_ens 5, Adam."""
    from vihmc.data import deeponet_problem
    from vihmc.vi import ELBO, BatchEngines, Bayesian_DeepONet, train_model
    prob = deeponet_problem(seed=3, n=256)
    grid = prob.trunk_in[0]
    priors = {"prior_mu": 0, "prior_sigma": 0.1, "posterior_mu_initial": (0, 0.1), "posterior_rho_initial": (-5, 0.1)}
    torch.manual_seed(7)
    m = Bayesian_DeepONet(priors, 100, 100, 101, 5, 9, 9, 100, "tanh", 0, 0, impose_bc=True).to(cuda_device)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    loader = [(torch.from_numpy(prob.branch_in[b:b + 128]), torch.from_numpy(np.broadcast_to(grid, (128,) + grid.shape)),
               torch.from_numpy(prob.y[b:b + 128])) for b in (0, 128)]
    eng = BatchEngines(m.spec, grid, 1.0, 5, cuda_device)
    try:
        train_model(loader[:1], m, ELBO(), opt, 1000 * grid.shape[0], 2, 5, 1.0, engines=eng)   # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        l = train_model(loader, m, ELBO(), opt, 1000 * grid.shape[0], 2, 5, 1.0, engines=eng)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 2
        print(f"VI training step (B=128, P=10201, num_ens=5, D=172401): {dt * 1e3:.1f} ms, loss {l:.1f}")
        assert np.isfinite(l)
    finally:
        eng.close()


def test_run_end_to_end_writes_artefacts(tmp_path, cuda_device):
    """vi.run (main_VI_deeponet.run) for two epochs on a small synthetic Burgers problem, then the
    sensitivity step on the exported posterior: the artefact files VI-HMC loads, in their formats."""
    from types import SimpleNamespace
    from vihmc import configs, sensitivity as S, vi
    from vihmc.data import deeponet_problem, load_vi_artefacts
    cfg = configs.load("burgers_vi", epochs=2, N_train=16, N_valid=8, batch_size=8, num_ens=2,
                       save_loc=str(tmp_path), uid="t", width_branch=20, width_trunk=20, output_neurons=20,
                       branch_depth=3, trunk_depth=3, in_branch=11)
    spec_like = SimpleNamespace(width_branch=20, width_trunk=20, in_branch=11, in_trunk=5, depth_branch=3,
                                depth_trunk=3, activation="tanh", output_neurons=20, impose_bc=True)
    from vihmc.layout import DeepONetSpec
    spec = DeepONetSpec(**vars(spec_like))
    prob = deeponet_problem(seed=1, n=24, nt=6, nx=7, spec=spec)
    grid = prob.trunk_in[0]
    P = grid.shape[0]
    cfg.p = P
    tr = vi.BurgersDataSet(prob.branch_in[:16], grid, prob.y[:16], P, seed=0)
    va = vi.BurgersDataSet(prob.branch_in[16:], grid, prob.y[16:], P, seed=1)
    tl = torch.utils.data.DataLoader(tr, batch_size=8, shuffle=True)
    vl = torch.utils.data.DataLoader(va, batch_size=8)
    torch.manual_seed(0)
    model, metrics = vi.run(cfg, tl, vl, 16 * P, 8 * P, grid, device=cuda_device, log=lambda s: None)
    assert len(metrics) == 2 and all(np.isfinite(m).all() for m in np.asarray(metrics))
    cfg_n = configs.load("burgers_vi", epochs=2, N_train=16, N_valid=8, batch_size=8, num_ens=2, width_branch=20,
                         width_trunk=20, output_neurons=20, branch_depth=3, trunk_depth=3, in_branch=11,
                         learn_noise=True, save_loc=None)
    cfg_n.p = P
    _, mn = vi.run(cfg_n, tl, vl, 16 * P, 8 * P, grid, device=cuda_device, log=lambda s: None)
    mn = np.asarray(mn)
    assert mn.shape == (2, 5) and np.isfinite(mn).all() and (mn[:, 4] > 0).all()      # 5th entry: exp(noise_param)
    mu = torch.load(f"{tmp_path}/means_flattened_t", weights_only=True)
    sd = torch.load(f"{tmp_path}/stds_flattened_t", weights_only=True)
    assert mu.shape == (spec.n_params,) and sd.shape == mu.shape and bool((sd > 0).all())
    pts = S.sample_points(8, P, 10, seed=2)
    scores = S.sensitivity_scores(spec, prob.branch_in[16:], grid, pts, mu, sd, device=cuda_device)
    ind = S.select_indices(scores, 0.9)
    from vihmc.data import save_vi_artefacts
    save_vi_artefacts(str(tmp_path), "t2", mu.numpy(), sd.numpy(), ind)
    m2, s2, i2 = load_vi_artefacts(str(tmp_path), "t2")
    assert np.array_equal(i2, ind) and np.all(np.diff(i2) > 0) and i2.size > 0

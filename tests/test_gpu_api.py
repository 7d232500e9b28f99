"""The reference-compatible surface on the GPU: define_model_log_prob closures (autograd), predict_model,
hamiltorch-style sample() with the closure, the split integrator, and the posterior-predictive mean
criterion (north star: within 1e-4 relative L2 of the reference)."""
import numpy as np
import pytest
import torch

from goldens import bnn_case, deeponet_case, load, spec_of
from oracle import hamiltorch_ref as HR
from oracle.bnn_ref import TorchBNNRef, mlp_layout
from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout

pytestmark = pytest.mark.gpu


def _layout(spec):
    return deeponet_layout(spec.in_branch, spec.width_branch, spec.depth_branch, spec.in_trunk, spec.width_trunk,
                           spec.depth_trunk, spec.out)


def _cfg(tmp_path, c):
    from vihmc import configs
    from vihmc.data import save_vi_artefacts
    save_vi_artefacts(str(tmp_path), "g", c.prob.mu, c.prob.sigma, c.prob.grad_ind)
    return configs.load("burgers_vi_hmc", prior_file=str(tmp_path), prior_uid="g",
                        branch_depth=c.spec.depth_branch, trunk_depth=c.spec.depth_trunk)


def _tr(c):
    p = c.prob
    return torch.from_numpy(p.branch_in), torch.from_numpy(p.trunk_in), torch.from_numpy(p.y)


def test_deeponet_closure_autograd_and_predict(tmp_path, cuda_device):
    from vihmc.operator import define_model_log_prob, predict_model
    c = deeponet_case("deeponet_small")
    cfg = _cfg(tmp_path, c)
    f = define_model_log_prob(c.spec, "NLL", _tr(c), [torch.tensor(cfg.prior_var)], 1.0, device=cuda_device, cfg=cfg)
    for t, th in enumerate(c.thetas):
        p = torch.tensor(th, device=cuda_device).requires_grad_()
        lp = f(p)
        assert lp.dim() == 0
        g, = torch.autograd.grad(lp, p)
        ref = float(c.g[f"logp{t}"])
        assert abs(float(lp) - ref) <= 2e-5 * abs(ref) + 1e-3
        gr = c.g[f"grad{t}"]
        assert np.linalg.norm(g.cpu().numpy() - gr) <= 2e-4 * np.linalg.norm(gr)
    preds, lps = predict_model(c.spec, torch.tensor(np.stack(c.thetas), device=cuda_device), _tr(c), "NLL", 1.0,
                               [torch.tensor(cfg.prior_var)], cfg=cfg)
    assert preds.shape == (2,) + c.prob.y.shape and len(lps) == 2
    for t in range(2):
        pr = c.g[f"pred{t}"]
        np.testing.assert_allclose(preds[t].cpu().numpy(), pr, rtol=1e-4, atol=1e-4 * np.abs(pr).max())


def test_deeponet_sample_data_closure_matches_golden(tmp_path, cuda_device):
    """cfg.sample_data (main_VI_HMC_burgers.py:127-137): after random.seed(seed) the closure's three successive
    calls draw the reference's trunk rows (vihmc_plan_set_trunk_rows gathers them on the device) and give the
    reference's log-prob and gradient; the engine path draws the same rows per call; predict stays on the full
    grid; the fused trajectory is off while rows are redrawn per evaluation."""
    import random
    import parity
    from vihmc import configs
    from vihmc.data import save_vi_artefacts
    from vihmc.operator import define_model_log_prob
    from vihmc.samplers import EngineEvaluator
    g = load("deeponet_sampledata")
    spec = spec_of(g)
    save_vi_artefacts(str(tmp_path), "g", g["mu"], g["sigma"], g["grad_ind"])
    cfg = configs.load("burgers_vi_hmc", prior_file=str(tmp_path), prior_uid="g", branch_depth=3, trunk_depth=3,
                       sample_data=True, p=int(g["p"]), prior_var=float(g["prior_var"]))
    tr = (torch.from_numpy(g["branch_in"]), torch.from_numpy(g["trunk_in"]), torch.from_numpy(g["y"]))
    f = define_model_log_prob(spec, str(g["loss"]), tr, [torch.tensor(cfg.prior_var)], float(g["tau_out"]),
                              device=cuda_device, cfg=cfg)
    eng = f._vihmc_engine
    assert eng.P == int(g["p"]) and not EngineEvaluator(eng).fused_trajectory

    def check(lp, gr, t, how):
        ref, rg = float(g[f"logp{t}"]), np.asarray(g[f"grad{t}"], np.float64)
        parity.check("logp_rel", abs(lp - ref) / max(abs(ref), 1.0), f"{how} call{t}")
        gr = np.asarray(gr, np.float64)
        parity.check("grad_relnorm", np.linalg.norm(gr - rg) / np.linalg.norm(rg), f"{how} call{t}")

    random.seed(int(g["seed"]))
    for t in range(3):
        p = torch.tensor(g[f"theta{t}"], device=cuda_device).requires_grad_()
        lp = f(p)
        gr, = torch.autograd.grad(lp, p)
        check(float(lp), gr.cpu().numpy(), t, "closure")
    random.seed(int(g["seed"]))
    for t in range(3):
        lp, gr = eng.logp_grad(torch.tensor(g[f"theta{t}"], device=cuda_device)[None])
        check(float(lp[0]), gr[0].cpu().numpy(), t, "engine")
    with pytest.raises(RuntimeError):
        eng.trajectory(torch.zeros(1, eng.K, device=cuda_device), torch.zeros(1, eng.K, device=cuda_device),
                       torch.zeros(1, eng.K, device=cuda_device), 1e-3, 2)
    with pytest.raises(ValueError):
        eng.set_trunk_rows([0] * (eng.P - 1) + [g["trunk_in"].shape[1]])
    fp = define_model_log_prob(spec, str(g["loss"]), tr, [torch.tensor(cfg.prior_var)], float(g["tau_out"]),
                               predict=True, device=cuda_device, cfg=cfg)
    _, out = fp(torch.tensor(g["theta0"], device=cuda_device))
    assert tuple(out.shape) == g["y"].shape


def test_sample_with_closure_matches_scalar_reference(tmp_path, cuda_device):
    from vihmc.operator import define_model_log_prob
    from vihmc.samplers import sample
    c = deeponet_case("deeponet_small")
    cfg = _cfg(tmp_path, c)
    f = define_model_log_prob(c.spec, "NLL", _tr(c), [torch.tensor(cfg.prior_var)], 1.0, device=cuda_device, cfg=cfg)
    th0 = torch.tensor(c.thetas[0], device=cuda_device)
    out = sample(f, th0, num_samples=12, num_steps_per_sample=7, step_size=2e-3, rng="per_chain", seed=77,
                 verbose=True)
    p = c.prob
    ref_fn = TorchDeepONetRef(_layout(c.spec), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, 0.0, 0.1).log_prob
    ref = HR.sample(ref_fn, th0.cpu(), 12, 7, 2e-3, generator=torch.Generator().manual_seed(77))
    assert len(out) == len(ref)
    for a, b in zip(out, ref):
        torch.testing.assert_close(a.cpu(), b, rtol=0, atol=1e-4)


def test_split_integrator_full_parameter(cuda_device):
    """Operator_network/HMC/main_HMC_splitting.py: 2 data shards, full-parameter closures with
    prior_scale=2, Integrator.SPLITTING."""
    from vihmc.operator import define_split_model_log_prob
    from vihmc.samplers import Integrator, sample
    g = load("deeponet_split")
    spec = spec_of(g)
    shards = [(torch.from_numpy(g["branch_in"][4 * m:4 * m + 4]), torch.from_numpy(g["trunk_in"]),
               torch.from_numpy(g["y"][4 * m:4 * m + 4])) for m in range(2)]
    fns = define_split_model_log_prob(spec, "NLL", shards, 2, [torch.tensor(float(g["prior_var"]))], 1.0,
                                      device=cuda_device, verbose=False)
    th0 = torch.tensor(g["theta"], device=cuda_device)
    for m, f in enumerate(fns):
        lp = float(f(th0))
        ref = float(g[f"logp_shard{m}"])
        assert abs(lp - ref) <= 2e-5 * abs(ref) + 1e-3
    out = sample(fns, th0, num_samples=5, num_steps_per_sample=3, step_size=1e-3, integrator=Integrator.SPLITTING,
                 rng="per_chain", seed=5, verbose=True)
    lay = _layout(spec)
    refs = [TorchDeepONetRef(lay, *[s.numpy() for s in sh], None, np.arange(spec.n_params), 0.0, 0.1,
                             prior_scale=2.0, full=True).log_prob for sh in shards]
    ref = HR.sample(refs, th0.cpu(), 5, 3, 1e-3, integrator=HR.SPLITTING, generator=torch.Generator().manual_seed(5))
    assert len(out) == len(ref)
    for a, b in zip(out, ref):
        torch.testing.assert_close(a.cpu(), b, rtol=0, atol=1e-4)


def test_bnn_closure_and_hmc_regression_sample_model(cuda_device):
    from vihmc import bnn, configs
    c = bnn_case("bnn_hmc_regression")
    g = c.g
    cfg = configs.load("nn_hmc")
    model = bnn.get_model(cfg, True)
    x = torch.from_numpy(c.data["x_train"]).to(cuda_device)
    y = torch.from_numpy(c.data["y_train"]).to(cuda_device)
    sizes = [p.nelement() for p in model.parameters()]
    f = bnn.define_model_log_prob_hamiltorch(model, "regression", x, y, sizes, None, torch.ones(len(sizes)), 400.0,
                                             device=cuda_device)
    p = torch.tensor(c.thetas[1], device=cuda_device).requires_grad_()
    lp = f(p)
    assert lp.shape == (1,)
    gr, = torch.autograd.grad(lp.sum(), p)
    assert abs(float(lp) - float(g["logp1"])) <= 2e-5 * abs(float(g["logp1"])) + 1e-3
    assert np.linalg.norm(gr.cpu().numpy() - g["grad1"]) <= 2e-4 * np.linalg.norm(g["grad1"])
    torch.manual_seed(0)
    out = bnn.sample_model(model, x, y, torch.tensor(c.thetas[0], device=cuda_device), "regression", num_samples=6,
                           num_steps_per_sample=20, step_size=1e-4, tau_out=400.0, tau_list=torch.ones(len(sizes)),
                           verbose=True)
    assert len(out) == 6 and all(o.shape == (141,) for o in out)
    preds, lps = bnn.predict_model_hamiltorch(model, torch.stack(out), torch.from_numpy(c.data["x_val"]),
                                              torch.from_numpy(c.data["y_val"]), "regression", 400.0)
    assert preds.shape == (6, 300, 1) and len(lps) == 6


def test_posterior_predictive_mean_within_1em4(cuda_device):
    """North-star criterion on the reduced problem: the same seeded chains on the HIP engine and in
    the scalar reference sampler give posterior-predictive means within 1e-4 relative L2."""
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = deeponet_case("deeponet_small")
    p = c.prob
    eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, 0.0, 0.1,
                         max_chains=2, device=cuda_device)
    th0 = torch.tensor(c.thetas[0])
    S, burn = 30, 5
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(2, 1), S, 7, 2e-3,
                     rng=ChainRNG(2, th0.numel(), cuda_device, seeds=[3, 4]))
    mine = res.stacked()[:, burn:].reshape(-1, th0.numel())

    preds = torch.cat([eng.forward(mine[i:i + 2])[1] for i in range(0, mine.shape[0], 2)])
    mean_gpu = preds.mean(0).double().cpu().numpy()
    ref_fn = TorchDeepONetRef(_layout(c.spec), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, 0.0, 0.1)
    ref_samples = []
    for s in (3, 4):
        out = HR.sample(ref_fn.log_prob, th0, S, 7, 2e-3, generator=torch.Generator().manual_seed(s))
        ref_samples += out[burn:]
    ref_preds = np.stack([ref_fn.forward(t.numpy())[1] for t in ref_samples]).astype(np.float64)
    mean_ref = ref_preds.mean(0)
    rel = np.linalg.norm(mean_gpu - mean_ref) / np.linalg.norm(mean_ref)
    assert rel < 1e-4, rel

"""The rest of the reference surface on the GPU engine:

* Operator_network/HMC/NUTS_DeepOnets.py -- its full-parameter closure (per-tensor prior Normal(0, tau/2)) against
  the reference-generated golden, and Sampler.HMC_NUTS (dual-averaging step size during burn, :289-290) on
  the engine against the scalar hamiltorch restatement driving the reference's torch ops;
* config 3 (Neural_network/VI_HMC BNN, 64 chains over 8 GPUs): one GPU's share (8 chains) and all 64 chains
  in one launch, every chain against its seeded scalar reference run; HMC_NUTS with per-chain adaptation.

Tolerances as tests/test_gpu_sampler.py: identical accept sequences and step sizes, positions within 1e-4.
"""
import numpy as np
import pytest
import torch

from goldens import bnn_case, load, spec_of
from oracle import hamiltorch_ref as HR
from oracle.bnn_ref import TorchBNNRef, mlp_layout
from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout

pytestmark = pytest.mark.gpu


def _nuts_case(dev):
    from vihmc.operator import define_model_log_prob_nuts
    g = load("deeponet_nuts")
    spec = spec_of(g)
    tr = (torch.from_numpy(g["branch_in"]), torch.from_numpy(g["trunk_in"]), torch.from_numpy(g["y"]))
    f = define_model_log_prob_nuts(spec, str(g["loss"]), tr, list(g["sizes"]), None,
                                   [torch.tensor(float(t)) for t in g["taus"]], float(g["tau_out"]), device=dev)
    return g, spec, f


def test_nuts_closure_matches_reference(cuda_device):
    g, spec, f = _nuts_case(cuda_device)
    th = torch.tensor(g["theta"], device=cuda_device).requires_grad_()
    lp = f(th)
    gr, = torch.autograd.grad(lp, th)
    ref = float(g["logp"])
    assert abs(float(lp) - ref) <= 2e-5 * abs(ref) + 1e-3
    assert np.linalg.norm(gr.cpu().numpy() - g["grad"]) <= 2e-4 * np.linalg.norm(g["grad"])


def test_hmc_nuts_dual_averaging_on_engine(cuda_device):
    from vihmc.engine import prior_per_tensor
    from vihmc.samplers import Sampler, sample
    g, spec, f = _nuts_case(cuda_device)
    D = spec.n_params
    th0 = torch.tensor(g["theta"], device=cuda_device)
    out, eps = sample(f, th0, num_samples=14, num_steps_per_sample=5, step_size=1e-3, burn=6,
                      sampler=Sampler.HMC_NUTS, rng="per_chain", seed=21, debug=2, verbose=True)
    lay = deeponet_layout(spec.in_branch, spec.width_branch, spec.depth_branch, spec.in_trunk, spec.width_trunk,
                          spec.depth_trunk, spec.out)
    ps = prior_per_tensor(list(g["sizes"]), D, list(0.5 * g["taus"].astype(np.float64)))
    ref_fn = TorchDeepONetRef(lay, g["branch_in"], g["trunk_in"], g["y"], None, np.arange(D), 0.0, ps,
                              str(g["loss"]), float(g["tau_out"]), full=True).log_prob
    ref, st = HR.sample(ref_fn, th0.cpu(), 14, 5, 1e-3, burn=6, sampler=HR.HMC_NUTS,
                        generator=torch.Generator().manual_seed(21), return_stats=True)
    print(f"NUTS step sizes {st['step_sizes']}, final {eps}")
    assert eps == pytest.approx(st["step_sizes"][-1], rel=1e-5)
    assert len(out) == len(ref)
    for a, b in zip(out, ref):
        torch.testing.assert_close(a.cpu(), b, rtol=0, atol=1e-4)


def _bnn(C, dev):
    from vihmc.engine import MLPEngine
    c = bnn_case("bnn_vi_hmc")
    eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], c.g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=C, device=dev)
    ref = TorchBNNRef(mlp_layout(), c.data["x_train"], c.data["y_train"], c.g["mu"], c.idx,
                      prior_list=list(c.g["prior_var"]), loss=c.loss, tau_out=c.tau_out).log_prob
    return c, eng, ref


@pytest.mark.parametrize("C", [8, 64])
def test_bnn_config3_chains_each_match_scalar_reference(C, cuda_device):
    """Config 3's chains (8 = one GPU's share of 64; 64 = the whole job in one launch), seeds 1000 + c."""
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c, eng, ref = _bnn(C, cuda_device)
    th0 = torch.tensor(c.thetas[0])
    seeds = [1000 + i for i in range(C)]
    S, L, eps = 6, 20, 5e-4
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(C, 1), S, L, eps, burn=1,
                     rng=ChainRNG(C, th0.numel(), cuda_device, seeds=seeds))
    check = range(C) if C <= 8 else range(0, C, 7)          # every 7th chain of 64 against its scalar run
    for i in check:
        out, st = HR.sample(ref, th0, S, L, eps, burn=1, generator=torch.Generator().manual_seed(seeds[i]),
                            return_stats=True)
        assert res.accepted[i].cpu().tolist() == st["accepts"]
        mine = res.chain(i)
        assert len(mine) == len(out)
        for a, b in zip(mine, out):
            torch.testing.assert_close(a.cpu(), b, rtol=0, atol=1e-4)


def test_bnn_nuts_per_chain_adaptation(cuda_device):
    """HMC_NUTS with 4 chains: each chain adapts its own step size (host arithmetic per chain, as hamiltorch)."""
    from vihmc.samplers import ChainRNG, EngineEvaluator, Sampler, run_chains
    C = 4
    c, eng, ref = _bnn(C, cuda_device)
    th0 = torch.tensor(c.thetas[0])
    seeds = [50 + i for i in range(C)]
    S, L, eps, burn = 12, 10, 2e-3, 6
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(C, 1), S, L, eps, burn=burn, sampler=Sampler.HMC_NUTS,
                     rng=ChainRNG(C, th0.numel(), cuda_device, seeds=seeds))
    for i in range(C):
        out, st = HR.sample(ref, th0, S, L, eps, burn=burn, sampler=HR.HMC_NUTS,
                            generator=torch.Generator().manual_seed(seeds[i]), return_stats=True)
        assert res.step_size[i] == pytest.approx(st["step_sizes"][-1], rel=1e-5)
        assert res.accepted[i].cpu().tolist() == st["accepts"]
        for a, b in zip(res.chain(i), out):
            torch.testing.assert_close(a.cpu(), b, rtol=0, atol=1e-4)

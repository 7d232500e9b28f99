"""The bench's own sampler path on the GPU: DeepONet trajectories whose L - 1 interior leapfrog steps run the
Gram-form contraction (vihmc_trajectory / vihmc_grad on W = 100 plans with max_chains >= gram_min_chains = 4, the
default), against the scalar hamiltorch restatement driving the reference's own torch log-prob
(oracle/hamiltorch_ref.sample + TorchDeepONetRef, fp32 CPU) on identical per-chain RNG streams
(Operator_network/VI_HMC/my_make_func.py:79-82, main_VI_HMC_burgers.py:162-163 + SURVEY App. A.2).

* accept sequences (decisions inside the TAU_DECISION band may differ, tests/test_gpu_scale_parity.py), positions
  (recorded bound) and the posterior-predictive mean (rel-L2 < 1e-4, the north-star criterion);
* the fused trajectory == the step-by-step path (evaluator.grad on the interior points) bit for bit at C = 4;
* reversibility: forward trajectory, momentum negated, backward trajectory -> theta0 within rounding (the form
  assignment -- residual at the end points, Gram at the interior ones -- is symmetric under time reversal);
* a chain's samples do not depend on how many chains share its launch (the form is a plan property);
* an odd-width plan evaluated right after a W = 100 Gram plan in one process equals a fresh process bit for bit
  (the round-3 illegal-address record).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import parity
from goldens import deeponet_case
from oracle.deeponet_ref import TorchDeepONetRef
from test_gpu_scale_parity import _engine, _layout, _predictive_mean_rel_l2, _trajectory_parity

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _ref(c):
    p = c.prob
    return TorchDeepONetRef(_layout(c.spec), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd,
                            c.loss, c.tau_out)


@pytest.mark.parametrize("case,S,L,eps,burn", [("deeponet_refshape", 30, 7, 5e-3, 5),
                                               ("deeponet_burgers", 3, 7, 1e-4, 0)])
def test_gram_trajectories_vs_reference_sampler(case, S, L, eps, burn, cuda_device):
    """C = 4 chains on a max_chains = 4 plan with the default gram_min_chains: every trajectory's L - 1 interior
    evaluations ran the Gram form (plan counters), and each chain follows the oracle sampler on its seed."""
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = deeponet_case(case)
    C = 4
    seeds = [1000 + i for i in range(C)]
    eng = _engine(c, C, cuda_device)
    assert eng.get_option("gram_min_chains") == 4 and eng.get_option("gram") & 1
    th0 = torch.tensor(c.thetas[0])
    eng.option("gram_evals", 0)
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(C, 1), S, L, eps, burn=burn,
                     rng=ChainRNG(C, th0.numel(), cuda_device, seeds=seeds))
    n_calls, n_gram = eng.get_option("grad_evals"), eng.get_option("gram_evals")
    # 1 opening evaluation + S trajectories of L evaluations, of which the L - 1 interior ones in Gram form
    assert (n_calls, n_gram) == (1 + S * L, S * (L - 1)), (n_calls, n_gram)
    ref = _ref(c)
    aligned, min_margin = _trajectory_parity(res, ref.log_prob, th0, seeds, S, L, eps, burn)
    rate = float(res.accepted.float().mean())
    print(f"{case} (Gram interior steps, C = 4): acceptance {rate:.2f}, smallest reference margin {min_margin:.2e}, "
          f"chains fully aligned {[a[2] for a in aligned]}")
    if case == "deeponet_refshape":
        assert 0.3 < rate < 0.99                      # the accept decision is exercised
    else:
        assert all(a[2] for a in aligned), "full-shape chain diverged from the reference sampler"
    gpu_s = [t for a in aligned for t in a[0][1:]]
    ref_s = [t for a in aligned for t in a[1][1:]]
    rel = _predictive_mean_rel_l2(eng, ref, gpu_s, ref_s, cuda_device)
    print(f"{case} posterior-predictive mean over {len(gpu_s)} samples: rel L2 {rel:.2e}")
    parity.check("mean_rel_l2", rel, f"{case}, {len(gpu_s)} samples, Gram interior steps")


def test_gram_trajectory_reversible(cuda_device):
    """theta0 -> (theta_L, p_L) -> (theta_L, -p_L) -> (theta0', -p0'): recovered within rounding, with the Gram form
    on the interior points (and, for scale, with the residual form everywhere)."""
    c = deeponet_case("deeponet_refshape")
    C, L, eps = 4, 7, 5e-3
    K = len(c.thetas[0])
    rng = np.random.default_rng(21)
    th0 = torch.tensor(np.stack([c.thetas[0] + 0.01 * rng.standard_normal(K) * (i > 0) for i in range(C)]),
                       dtype=torch.float32, device=cuda_device)
    p0 = torch.tensor(rng.standard_normal((C, K)), dtype=torch.float32, device=cuda_device)
    errs = {}
    for form in ("gram", "residual"):
        eng = _engine(c, C, cuda_device)
        eng.option("gram", 1 if form == "gram" else 0)
        lp0, g0 = eng.logp_grad(th0)
        eng.option("gram_evals", 0)
        th1, p1, lp1, g1 = eng.trajectory(th0, p0, g0, eps, L)
        th2, p2, lp2, g2 = eng.trajectory(th1, -p1, g1, eps, L)
        assert eng.get_option("gram_evals") == (2 * (L - 1) if form == "gram" else 0)
        e_th = float((th2 - th0).abs().max())
        e_p = float((p2 + p0).abs().max())
        dH = float(((-lp1 + 0.5 * (p1 * p1).sum(1)) - (-lp0 + 0.5 * (p0 * p0).sum(1))).abs().max())
        moved = float((th1 - th0).abs().max())
        errs[form] = (e_th, e_p)
        print(f"{form}: |theta_back - theta0| {e_th:.2e} (trajectory moved {moved:.2e}), |p_back + p0| {e_p:.2e}, "
              f"|dH| forward {dH:.2e}")
        parity.check("pos_maxabs", e_th, f"{form}: reversed trajectory vs theta0")
        parity.check("mom_maxabs", e_p, f"{form}: reversed momentum vs -p0")
    # the Gram interior gradients cost no more reversibility than fp32 rounding of the residual form does
    assert errs["gram"][0] <= 4 * errs["residual"][0] + 1e-7, errs


@pytest.mark.parametrize("case", ["deeponet_refshape", "deeponet_burgers"])
def test_deeponet_sharding_independence_gram(case, cuda_device):
    """A chain's samples depend only on its seed: 4 chains on a max_chains = 4 plan vs 2 of them alone on the same
    plan (the Gram form runs in both: it is decided by the plan, not the call's chain count), bit for bit."""
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = deeponet_case(case)
    eng = _engine(c, 4, cuda_device)
    th0 = torch.tensor(c.thetas[0], device=cuda_device)
    K = th0.numel()
    S, L, eps = (6, 7, 5e-3) if case == "deeponet_refshape" else (2, 7, 1e-4)
    full = run_chains(EngineEvaluator(eng), th0[None].repeat(4, 1), S, L, eps,
                      rng=ChainRNG(4, K, cuda_device, seeds=[100, 101, 102, 103]))
    eng.option("gram_evals", 0)
    part = run_chains(EngineEvaluator(eng), th0[None].repeat(2, 1), S, L, eps,
                      rng=ChainRNG(2, K, cuda_device, seeds=[102, 103]))
    assert eng.get_option("gram_evals") == S * (L - 1)
    assert torch.equal(full.accepted[2:], part.accepted)
    assert torch.equal(full.stacked()[2:], part.stacked())
    assert torch.equal(full.logp_trace[2:], part.logp_trace)


_FRESH = r"""
import sys, numpy as np, torch
sys.path[:0] = [{root!r}, {root!r} + '/vi-hmc_amd', {root!r} + '/tests']
from goldens import deeponet_case
from vihmc.engine import DeepONetEngine, trunk_features
c = deeponet_case('deeponet_odd_full'); p = c.prob
eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd,
                     c.loss, c.tau_out, max_chains=2, device='cuda:0')
th = torch.tensor(np.stack(c.thetas), device='cuda:0')
lp, g = eng.logp_grad(th)
lpf, out = eng.forward(th)
np.savez({out!r}, lp=lp.cpu().numpy(), g=g.cpu().numpy(), lpf=lpf.cpu().numpy(), out=out.cpu().numpy())
"""


def test_odd_width_plan_after_gram_plan_matches_fresh_process(cuda_device, tmp_path):
    """Round-3 fault record: an odd-width plan (widths 37 / 21, N = 45, P = 63, full K) evaluated right
    after a W = 100 plan ran the Gram form on the same device equals the same evaluation in a fresh process."""
    from vihmc.engine import DeepONetEngine, trunk_features
    fresh = str(tmp_path / "fresh.npz")
    subprocess.run([sys.executable, "-c", _FRESH.format(root=ROOT, out=fresh)], check=True, timeout=300)
    ref = np.load(fresh)
    cb = deeponet_case("deeponet_burgers")
    big = _engine(cb, 4, cuda_device)
    thb = torch.tensor(np.stack([cb.thetas[0]] * 4), device=cuda_device)
    big.grad(thb)
    assert big.get_option("gram") & 2
    c = deeponet_case("deeponet_odd_full")
    p = c.prob
    eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                         c.prior_sd, c.loss, c.tau_out, max_chains=2, device=cuda_device)
    th = torch.tensor(np.stack(c.thetas), device=cuda_device)
    lp, g = eng.logp_grad(th)
    big.grad(thb)                                   # interleave a Gram evaluation between the odd plan's calls
    lpf, out = eng.forward(th)
    torch.cuda.synchronize()
    assert np.array_equal(lp.cpu().numpy(), ref["lp"]) and np.array_equal(g.cpu().numpy(), ref["g"])
    assert np.array_equal(lpf.cpu().numpy(), ref["lpf"]) and np.array_equal(out.cpu().numpy(), ref["out"])
    big.close()
    eng.close()


@pytest.mark.parametrize("case,C", [("deeponet_small", 2), ("deeponet_odd_full", 2), ("deeponet_refshape", 4),
                                    ("deeponet_burgers", 4), ("deeponet_burgers", 1)])
def test_no_out_of_bounds_writes_into_plan_buffers(case, C, cuda_device, monkeypatch):
    """Bounds audit (VIHMC_CANARY=1: a 4-KB 0xA5 tail behind every plan buffer): value, gradient, Gram-form gradient,
    forward and one fused trajectory on every golden geometry (odd widths 37 / 21, N = 45, P = 63 included) leave
    every tail intact."""
    from vihmc.engine import DeepONetEngine, trunk_features
    monkeypatch.setenv("VIHMC_CANARY", "1")
    c = deeponet_case(case)
    p = c.prob
    eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                         c.prior_sd, c.loss, c.tau_out, max_chains=C, device=cuda_device)
    monkeypatch.delenv("VIHMC_CANARY")
    eng.option("gram_min_chains", 1)
    n = len(c.thetas)
    th = torch.tensor(np.stack([c.thetas[i % n] for i in range(C)]), device=cuda_device)
    lp, g = eng.logp_grad(th)
    eng.logp(th)
    eng.grad(th)
    eng.forward(th)
    pm = torch.randn(th.shape, generator=torch.Generator().manual_seed(1)).to(cuda_device)
    eng.trajectory(th, pm, g, 1e-5, 3)
    assert eng.check_canaries() == 0
    eng.close()


def test_no_out_of_bounds_writes_bnn(cuda_device, monkeypatch):
    from goldens import bnn_case
    from vihmc.engine import MLPEngine
    monkeypatch.setenv("VIHMC_CANARY", "1")
    c = bnn_case("bnn_vi_hmc")
    g = c.g
    eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=3, device=cuda_device)
    monkeypatch.delenv("VIHMC_CANARY")
    th = torch.tensor(np.stack([c.thetas[0]] * 3), device=cuda_device)
    lp, gr = eng.logp_grad(th)
    eng.forward(th)
    eng.trajectory(th, torch.ones_like(th), gr, 1e-4, 5)
    assert eng.check_canaries() == 0

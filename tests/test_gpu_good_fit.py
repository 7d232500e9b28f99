"""The posterior the reference actually samples: the reference starts HMC at a TRAINED VI mean and
freezes the other weights there (Operator_network/VI_HMC/main_VI_HMC_burgers.py:63-65,278-283), so the network fits
the data to its noise. Here: deeponet_problem(noise=1e-3, mu_noise=0) -- frozen weights = the generator of the data,
sum r^2 / sum y^2 ~ 1.5e-3 at mu -- at the bench geometry (Burgers N = 1000, P = 10,201, K = 17,240, a max_chains = 16
plan, L = 7, eps = 1e-4, prior N(0, 0.1), the default options), 16 chains from mu on distinct seeds:

* every trajectory's L - 1 interior evaluations run the (centred) Gram form on all 16 chains: its fit guard compares
  sum r^2 with sum y~^2, y~ = y - the output at the centre (the frozen weights), ~1 here;
* chains 0, 7 and 15 against the scalar hamiltorch restatement driving the reference's torch log-prob
  (oracle/hamiltorch_ref.sample + TorchDeepONetRef, fp32 CPU) on their seeds: accept decisions (outside TAU_DECISION),
  positions, the posterior-predictive mean (rel-L2, the north-star criterion), with recorded bounds (tests/parity.py).
"""
import numpy as np
import pytest
import torch

import parity
from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout
from test_gpu_scale_parity import _predictive_mean_rel_l2, _trajectory_parity

pytestmark = pytest.mark.gpu

C, S, L, EPS = 16, 10, 7, 1e-4
CHECKED = [0, 7, 15]


@pytest.fixture(scope="module")
def good_fit_run(cuda_device):
    from vihmc.data import deeponet_problem
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.layout import DeepONetSpec
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    spec = DeepONetSpec()
    p = deeponet_problem(seed=0, noise=1e-3, mu_noise=0.0)
    eng = DeepONetEngine(spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, 0.0, 0.1, "NLL", 1.0,
                         max_chains=C, device=cuda_device)
    assert eng.get_option("gram_center") == 1 and eng.get_option("gram_guard") > 0 and eng.get_option("gram_active")
    th0 = torch.tensor(p.mu[p.grad_ind])[None].repeat(C, 1)
    seeds = [4000 + i for i in range(C)]
    eng.option("gram_evals", 0)
    res = run_chains(EngineEvaluator(eng), th0.to(cuda_device), S, L, EPS,
                     rng=ChainRNG(C, th0.shape[1], cuda_device, seeds=seeds))
    counters = {k: eng.get_option(k) for k in ("grad_evals", "gram_evals", "gram_chain_evals")}
    ref = TorchDeepONetRef(deeponet_layout(), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, 0.0, 0.1, "NLL", 1.0)
    yield p, eng, th0, seeds, res, counters, ref
    eng.close()


def test_good_fit_gram_counters(good_fit_run):
    _, _, _, _, res, n, _ = good_fit_run
    assert n["grad_evals"] == 1 + S * L, n
    assert n["gram_evals"] == S * (L - 1), n
    assert n["gram_chain_evals"] == C * S * (L - 1), n
    last = torch.stack([res.chain(i)[-1] for i in range(C)])
    assert torch.unique(last, dim=0).shape[0] == C


@pytest.mark.parametrize("chain", CHECKED)
def test_good_fit_trajectory_vs_reference_sampler(good_fit_run, chain, cuda_device):
    p, eng, th0, seeds, res, _, ref = good_fit_run
    aligned, min_margin = _trajectory_parity(res, ref.log_prob, th0, [seeds[chain]], S, L, EPS, chains=[chain])
    gpu_s, ref_s, full = aligned[0]
    acc = res.accepted[chain].cpu().tolist()
    print(f"chain {chain}: accepts {acc}, smallest reference margin {min_margin:.2e}, aligned over all {S}: {full}")
    assert full, "a good-fit trajectory diverged from the reference sampler"
    assert sum(acc) >= S // 2
    rel = _predictive_mean_rel_l2(eng, ref, gpu_s[1:], ref_s[1:], cuda_device)
    print(f"chain {chain}: posterior-predictive mean over {len(gpu_s) - 1} samples: rel L2 {rel:.2e}")
    parity.check("mean_rel_l2", rel, f"good fit, C=16, chain {chain}")

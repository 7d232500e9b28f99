"""The bench's timed path exactly as it runs (bench.py: Burgers shape N = 1000, P = 10,201, K = 17,240, 16 chains on a
max_chains = 16 plan, L = 7, eps = 1e-4, the default gram_min_chains / gram_guard), with 16 DISTINCT chains -- the
round-4 Gram race (one Gt element written twice from mirrored diagonal tiles) showed only with distinct
chains, and the C = 16 geometry (8 T_b slabs per chain, St = 8, no T_t split) is the bench's own:

* trajectories: every trajectory's L - 1 interior evaluations in the Gram form on all 16 chains (plan counters);
  chains 0, 7 and 15 against the scalar hamiltorch restatement driving the reference's torch log-prob
  (oracle/hamiltorch_ref.sample + TorchDeepONetRef, fp32 CPU) on their seeds: accept decisions (outside the
  TAU_DECISION band), positions, and the posterior-predictive mean (rel-L2, the north-star criterion);
* gradients: the C = 16 Gram-form gradient of every chain against the fp64 oracle (oracle/deeponet_ref.np_logp_grad).

Reference: Operator_network/VI_HMC/my_make_func.py:44-83 (the forward and, through autograd, its backward),
main_VI_HMC_burgers.py:86-178 (the closure), :286-287 (the sampler call); hamiltorch semantics SURVEY App. A.
"""
import numpy as np
import pytest
import torch

import parity
from goldens import deeponet_case
from oracle.deeponet_ref import deeponet_layout, np_logp_grad
from test_gpu_scale_parity import _engine, _predictive_mean_rel_l2, _trajectory_parity
from test_gpu_gram_traj import _ref

pytestmark = pytest.mark.gpu

C, S, L, EPS = 16, 12, 7, 1e-4
CHECKED = [0, 7, 15]


def _thetas(c):
    """16 distinct starts: the golden theta + 0.01 N(0, 1) per chain (seeded)."""
    th0 = np.asarray(c.thetas[0], np.float32)
    rng = np.random.default_rng(2024)
    return np.stack([th0 + (0.01 * rng.standard_normal(th0.size)).astype(np.float32) for _ in range(C)])


@pytest.fixture(scope="module")
def bench_run(cuda_device):
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = deeponet_case("deeponet_burgers")
    eng = _engine(c, C, cuda_device)
    assert eng.get_option("gram_min_chains") == 4 and eng.get_option("gram") & 1 and eng.get_option("gram_guard") > 0
    assert all(eng.get_option(k) == 1 for k in ("fwd_bf16x6", "contract_bf16x6", "bwd_bf16x6"))
    th0 = torch.tensor(_thetas(c))
    seeds = [1000 + i for i in range(C)]
    eng.option("gram_evals", 0)
    res = run_chains(EngineEvaluator(eng), th0.to(cuda_device), S, L, EPS,
                     rng=ChainRNG(C, th0.shape[1], cuda_device, seeds=seeds))
    counters = {k: eng.get_option(k) for k in ("grad_evals", "gram_evals", "gram_chain_evals")}
    yield c, eng, th0, seeds, res, counters
    eng.close()


def test_bench_geometry_gram_counters(bench_run):
    """1 opening evaluation + S trajectories of L evaluations; the L - 1 interior ones in the Gram form, for every
    one of the 16 chains (none guarded: their fits are far above the guard threshold)."""
    _, _, _, _, res, n = bench_run
    assert n["grad_evals"] == 1 + S * L, n
    assert n["gram_evals"] == S * (L - 1), n
    assert n["gram_chain_evals"] == C * S * (L - 1), n
    assert res.samples.shape[0] == C
    # distinct chains stay distinct (no cross-chain write)
    last = torch.stack([res.chain(i)[-1] for i in range(C)])
    assert torch.unique(last, dim=0).shape[0] == C


@pytest.mark.parametrize("chain", CHECKED)
def test_bench_geometry_trajectory_vs_reference_sampler(bench_run, chain, cuda_device):
    c, eng, th0, seeds, res, _ = bench_run
    ref = _ref(c)
    aligned, min_margin = _trajectory_parity(res, ref.log_prob, th0, [seeds[chain]], S, L, EPS, chains=[chain])
    gpu_s, ref_s, full = aligned[0]
    acc = res.accepted[chain].cpu().tolist()
    print(f"chain {chain}: accepts {acc}, smallest reference margin {min_margin:.2e}, aligned over all {S}: {full}")
    assert full, "a 16-chain bench-geometry trajectory diverged from the reference sampler"
    assert sum(acc) >= S // 2                                   # the chain moves (eps = 1e-4 accepts ~always)
    rel = _predictive_mean_rel_l2(eng, ref, gpu_s[1:], ref_s[1:], cuda_device)
    print(f"chain {chain}: posterior-predictive mean over {len(gpu_s) - 1} samples: rel L2 {rel:.2e}")
    parity.check("mean_rel_l2", rel, f"C=16 bench geometry, chain {chain}")


def test_bench_geometry_gram_grad_vs_fp64_oracle(cuda_device):
    """The C = 16 Gram-form gradient (k_gram_a / k_gram_b at 8 T_b slabs, St = 8) on 16 distinct thetas against the
    fp64 oracle, every chain."""
    c = deeponet_case("deeponet_burgers")
    p, s = c.prob, c.spec
    eng = _engine(c, C, cuda_device)
    th = _thetas(c)
    eng.option("gram_evals", 0)
    g = eng.grad(torch.tensor(th, device=cuda_device)).cpu().numpy()
    assert eng.get_option("gram") & 2 and eng.get_option("gram_chain_evals") == C
    lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk,
                          s.out)
    for i in range(C):
        _, rg, _ = np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, th[i], c.prior_mu, c.prior_sd,
                                c.loss, c.tau_out)
        parity.check("grad_relnorm", np.linalg.norm(g[i] - rg) / np.linalg.norm(rg), f"chain {i}")
        parity.check("grad_elem", np.abs(g[i] - rg).max() / np.abs(rg).max(), f"chain {i}")
    eng.close()

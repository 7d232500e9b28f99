"""Batched GPU sampler on the HIP engine vs the scalar hamiltorch restatement on the CPU with the
reference's own torch log-prob (oracle), on identical per-chain RNG streams.

Tolerance statement: the engine's log-prob differs from the CPU reference by fp32 summation order
(~1e-6 relative), so trajectories agree to ~1e-5 absolute over the first samples and accept
decisions agree except where |rho - log u| falls below that drift; the test requires identical
accept sequences for the first 15 samples and positions within 1e-4 (max-abs).
"""
import numpy as np
import pytest
import torch

import parity
from goldens import bnn_case, deeponet_case
from oracle import hamiltorch_ref as HR
from oracle.bnn_ref import TorchBNNRef, mlp_layout
from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout

pytestmark = pytest.mark.gpu


# Identical accept sequences need every reference decision clear of the Hamiltonian's fp32 rounding: at the BNN's
# |H| ~ 7.5e4 one ulp is 0.0078, and a margin rho - log u inside a few ulps is decided by summation order (the
# reference's own CPU dot products move it by an ulp between machines: profiles/r05am_accept_margin.txt)
MARGIN_FLOOR = 0.015


def _compare(res, fn, th0, seeds, S, L, eps, burn=0, atol=1e-4, inv_mass=None):
    for c, s in enumerate(seeds):
        g = torch.Generator().manual_seed(s)
        out, st = HR.sample(fn, th0, S, L, eps, burn=burn, generator=g, return_stats=True, inv_mass=inv_mass)
        margin = min(abs(a - b) for a, b in zip(st["rhos"], st["logus"]))
        assert margin > MARGIN_FLOOR, f"seed {s}: a borderline accept decision ({margin:.2e}); pick other seeds"
        assert res.accepted[c].cpu().tolist() == st["accepts"]
        mine = [t.cpu() for t in res.chain(c)]
        assert len(mine) == len(out)
        parity.check("pos_maxabs", max(float((a - b).abs().max()) for a, b in zip(mine, out)),
                     f"chain {c}, {len(out)} samples")


def test_bnn_chains_gpu_vs_scalar_reference(cuda_device):
    from vihmc.engine import MLPEngine
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = bnn_case("bnn_vi_hmc")
    g = c.g
    eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=3, device=cuda_device)
    th0 = torch.tensor(c.thetas[0])
    seeds = [1, 2, 3]
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(3, 1), 15, 10, 5e-4, burn=2,
                     rng=ChainRNG(3, th0.numel(), cuda_device, seeds=seeds))
    fn = TorchBNNRef(mlp_layout(), c.data["x_train"], c.data["y_train"], g["mu"], c.idx,
                     prior_list=list(g["prior_var"]), loss=c.loss, tau_out=c.tau_out).log_prob
    _compare(res, fn, th0, seeds, 15, 10, 5e-4, burn=2)


def test_bnn_config3_eight_chains_vs_scalar_reference(cuda_device):
    """Config 3's per-GPU geometry (BASELINE.json: 64 BNN chains over 8 GPUs = 8 chains per plan; Neural_network/VI_HMC/
    main_VI_HMC.py:458-460 runs its chains one after the other): an 8-chain plan on the fused trajectory kernel
    (k_mlp_traj_bnn, one wave per chain) at the reference's L = 196, eps = 5e-4, 8 seeds, 6 samples with one burn-in
    iteration, each chain against the scalar hamiltorch restatement with the reference's torch log-prob: identical
    accept sequences, positions within the recorded bound. Seeds 100..112 minus 101 (its sample 2 decision lies 0.004
    from the uniform: below MARGIN_FLOOR) and 108..111 (all-accept duplicates), chosen on the CPU oracle alone."""
    from vihmc.engine import MLPEngine
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = bnn_case("bnn_vi_hmc")
    g = c.g
    C = 8
    eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=C, device=cuda_device)
    ev = EngineEvaluator(eng)
    assert ev.fused_trajectory and eng.get_option("mlp_fast")
    th0 = torch.tensor(c.thetas[0])
    seeds = [100, 102, 103, 104, 105, 106, 107, 112]
    res = run_chains(ev, th0[None].repeat(C, 1), 6, 196, 5e-4, burn=1, rng=ChainRNG(C, th0.numel(), cuda_device,
                                                                                    seeds=seeds))
    fn = TorchBNNRef(mlp_layout(), c.data["x_train"], c.data["y_train"], g["mu"], c.idx,
                     prior_list=list(g["prior_var"]), loss=c.loss, tau_out=c.tau_out).log_prob
    # 980 leapfrog steps per chain: the fp32 rounding differences between the engine's and the CPU's dot products grow
    # along the trajectory (the BNN likelihood's precision 400 makes it stiff), so the positions carry their own bound;
    # the accept decisions must agree exactly
    drift = []
    for ci, sd in enumerate(seeds):
        out, st = HR.sample(fn, th0, 6, 196, 5e-4, burn=1, generator=torch.Generator().manual_seed(sd),
                            return_stats=True)
        margin = min(abs(a - b) for a, b in zip(st["rhos"], st["logus"]))
        assert margin > MARGIN_FLOOR, f"seed {sd}: a borderline accept decision ({margin:.2e})"
        assert res.accepted[ci].cpu().tolist() == st["accepts"], (ci, sd)
        mine = [t.cpu() for t in res.chain(ci)]
        assert len(mine) == len(out)
        drift.append(max(float((a - b).abs().max()) for a, b in zip(mine, out)))
    print("position drift per chain:", [f"{d:.2e}" for d in drift])
    parity.check("pos_maxabs", max(drift), f"8 chains x 6 samples x L = 196")
    assert 0 < float(res.accepted.float().mean()) < 1


def test_deeponet_chains_gpu_vs_scalar_reference(cuda_device):
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = deeponet_case("deeponet_small")
    p = c.prob
    eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                         c.prior_sd, c.loss, c.tau_out, max_chains=2, device=cuda_device)
    th0 = torch.tensor(c.thetas[0])
    seeds = [10, 11]
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(2, 1), 15, 7, 2e-3,
                     rng=ChainRNG(2, th0.numel(), cuda_device, seeds=seeds))
    lay = deeponet_layout(c.spec.in_branch, c.spec.width_branch, c.spec.depth_branch, c.spec.in_trunk,
                          c.spec.width_trunk, c.spec.depth_trunk, c.spec.out)
    fn = TorchDeepONetRef(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd, c.loss,
                          c.tau_out).log_prob
    _compare(res, fn, th0, seeds, 15, 7, 2e-3)
    assert res.n_grad_evals == 2 * (1 + 15 * 7)


@pytest.mark.parametrize("kind", ["deeponet", "bnn"])
def test_inv_mass_fused_trajectory_vs_scalar_reference(kind, cuda_device):
    """The VI-preconditioned mass matrix (diagonal inv_mass = sigma_VI^2 of the sampled coordinates, rescaled to
    O(1)) on the engine's fused trajectory path vs the scalar hamiltorch restatement with the same mass and the
    reference's own torch log-prob: identical accept sequences, positions within the recorded bound. The synthetic
    DeepONet artefacts have a constant sigma_VI, so a seeded spread in [0.5, 2] multiplies it (every coordinate
    scaled differently)."""
    from vihmc.engine import DeepONetEngine, MLPEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    if kind == "deeponet":
        c = deeponet_case("deeponet_small")
        p = c.prob
        eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                             c.prior_sd, c.loss, c.tau_out, max_chains=2, device=cuda_device)
        sig = np.asarray(p.sigma, np.float64)[p.grad_ind]
        lay = deeponet_layout(c.spec.in_branch, c.spec.width_branch, c.spec.depth_branch, c.spec.in_trunk,
                              c.spec.width_trunk, c.spec.depth_trunk, c.spec.out)
        fn = TorchDeepONetRef(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd, c.loss,
                              c.tau_out).log_prob
        S, L, eps, seeds = 12, 7, 2e-3, [30, 31]
    else:
        c = bnn_case("bnn_vi_hmc")
        g = c.g
        eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                        c.tau_out, max_chains=2, device=cuda_device)
        sig = np.abs(np.asarray(g["mu"], np.float64)[c.idx]) * 0.1 + 0.01
        fn = TorchBNNRef(mlp_layout(), c.data["x_train"], c.data["y_train"], g["mu"], c.idx,
                         prior_list=list(g["prior_var"]), loss=c.loss, tau_out=c.tau_out).log_prob
        S, L, eps, seeds = 12, 20, 5e-4, [42, 43]       # 40, 41: seed 41's step 5 is borderline (5e-5 / 0.0078)
    spread = np.exp(np.random.default_rng(8).uniform(-np.log(2.0), np.log(2.0), sig.size))
    inv_mass = torch.tensor(sig ** 2 / np.mean(sig ** 2) * spread, dtype=torch.float32)
    assert EngineEvaluator(eng).fused_trajectory
    th0 = torch.tensor(c.thetas[0])
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(2, 1), S, L, eps, inv_mass=inv_mass,
                     rng=ChainRNG(2, th0.numel(), cuda_device, seeds=seeds))
    _compare(res, fn, th0, seeds, S, L, eps, inv_mass=inv_mass)
    assert 0 < float(res.accepted.float().mean())


def test_sharding_independence(cuda_device):
    """A chain's samples depend only on its seed, not on which/how many chains share the launch."""
    from vihmc.engine import MLPEngine
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = bnn_case("bnn_vi_hmc")
    g = c.g
    eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=4, device=cuda_device)
    th0 = torch.tensor(c.thetas[0], device=cuda_device)
    K = th0.numel()
    full = run_chains(EngineEvaluator(eng), th0[None].repeat(4, 1), 8, 6, 5e-4,
                      rng=ChainRNG(4, K, cuda_device, seeds=[100, 101, 102, 103]))
    part = run_chains(EngineEvaluator(eng), th0[None].repeat(2, 1), 8, 6, 5e-4,
                      rng=ChainRNG(2, K, cuda_device, seeds=[102, 103]))
    assert torch.equal(full.stacked()[2:], part.stacked())


@pytest.mark.parametrize("variant,case,fuse_scatter,C", [("hmc", "deeponet_small", 1, 3),
                                                         ("inv_mass", "deeponet_small", 1, 3),
                                                         ("nuts", "deeponet_small", 1, 3),
                                                         ("inv_mass", "deeponet_refshape", 1, 2),
                                                         ("hmc", "deeponet_refshape", 0, 2),
                                                         ("hmc", "deeponet_refshape", 1, 4),
                                                         ("nuts", "deeponet_refshape", 1, 4)])
def test_deeponet_fused_trajectory_bitwise_equals_stepwise(variant, case, fuse_scatter, C, cuda_device):
    """vihmc_trajectory on a DeepONet plan (leapfrog updates fused into the gradient gather) == L separate
    evaluations driven by the torch elementwise updates, bit for bit: positions, accepts, log-probs, step sizes.
    deeponet_refshape is width 100: the bf16x6 fused forward, the weight images kept current by the scatter and by
    the leapfrog's own scatter in k_leap_open / k_gather_prior<LEAP> (fuse_scatter = 1) or by k_scatter (0). At
    C = 4 (max_chains 4 >= gram_min_chains) both paths run the interior steps in Gram form (counters checked)."""
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, Sampler, run_chains
    c = deeponet_case(case)
    p = c.prob
    th0 = torch.tensor(c.thetas[0])
    kw = dict(burn=2)
    if variant == "inv_mass":
        kw["inv_mass"] = torch.linspace(0.5, 1.5, th0.numel())
    if variant == "nuts":
        kw.update(sampler=Sampler.HMC_NUTS, burn=4)
    out = []
    for fused in (True, False):
        eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                             c.prior_sd, c.loss, c.tau_out, max_chains=C, device=cuda_device)
        eng.fused_trajectory = fused
        eng.option("fuse_scatter", fuse_scatter)
        S, L, eps = (8, 7, 2e-3) if case == "deeponet_small" else (5, 3, 5e-3)
        eng.option("gram_evals", 0)
        out.append(run_chains(EngineEvaluator(eng), th0[None].repeat(C, 1), S, L, eps,
                              rng=ChainRNG(C, th0.numel(), cuda_device, seeds=[20 + i for i in range(C)]), **kw))
        n_gram = eng.get_option("gram_evals")
        assert (n_gram == S * (L - 1)) if (C >= 4 and case == "deeponet_refshape") else n_gram == 0, n_gram
    a, b = out
    assert torch.equal(a.accepted, b.accepted)
    assert torch.equal(a.counts, b.counts)
    assert torch.equal(a.samples[:, :int(a.counts.max())], b.samples[:, :int(b.counts.max())])
    assert torch.equal(a.logp_trace, b.logp_trace)
    assert a.step_size == b.step_size
    assert a.n_grad_evals == b.n_grad_evals


@pytest.mark.parametrize("variant", ["hmc", "inv_mass", "nuts"])
def test_bnn_fused_trajectory_bitwise_equals_stepwise(variant, cuda_device):
    """vihmc_mlp_trajectory (one launch per trajectory) == L separate evaluations driven by the torch
    elementwise updates, bit for bit: positions, accept decisions, log-probs and step sizes."""
    from vihmc.engine import MLPEngine
    from vihmc.samplers import ChainRNG, EngineEvaluator, Sampler, run_chains
    c = bnn_case("bnn_vi_hmc")
    g = c.g
    C = 5
    th0 = torch.tensor(c.thetas[0])
    kw = dict(burn=3)
    if variant == "inv_mass":
        kw["inv_mass"] = torch.linspace(0.5, 1.5, th0.numel())
    if variant == "nuts":
        kw.update(sampler=Sampler.HMC_NUTS, burn=5)
    out = []
    for fused in (True, False):
        eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                        c.tau_out, max_chains=C, device=cuda_device)
        eng.fused_trajectory = fused
        out.append(run_chains(EngineEvaluator(eng), th0[None].repeat(C, 1), 12, 25, 1e-3,
                              rng=ChainRNG(C, th0.numel(), cuda_device, seeds=[7 + i for i in range(C)]), **kw))
    a, b = out
    assert torch.equal(a.accepted, b.accepted)
    assert torch.equal(a.counts, b.counts)
    assert torch.equal(a.samples[:, :int(a.counts.max())], b.samples[:, :int(b.counts.max())])
    assert torch.equal(a.logp_trace, b.logp_trace)
    assert a.step_size == b.step_size
    assert 0 < float(a.accepted.float().mean()) < 1 or variant != "hmc"


def test_bnn_register_kernels_match_generic_kernels(cuda_device):
    """The register-resident BNN kernels (vihmc_bnn.hip: weights in registers, dW as two fp32 MFMA tiles) against
    the generic LDS kernels (plan option mlp_fast = 0) on the same plan: evaluation (logp, gradient, predictions)
    and a whole fused trajectory. Both are fp32 computations that differ only in the order of the row sums."""
    from vihmc.engine import MLPEngine
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = bnn_case("bnn_vi_hmc")
    g = c.g
    C = 4
    eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=C, device=cuda_device)
    assert eng.get_option("mlp_fast") == 1
    rng = np.random.default_rng(3)
    th = torch.tensor(np.stack([c.thetas[0] + 0.05 * rng.standard_normal(c.thetas[0].size).astype(np.float32)
                                for _ in range(C)]), device=cuda_device)
    out = {}
    for fast in (1, 0):
        eng.option("mlp_fast", fast)
        lp, gr = eng.logp_grad(th)
        out[fast] = (lp.double().cpu().numpy(), gr.double().cpu().numpy())
    dlp = np.abs(out[1][0] - out[0][0]) / np.maximum(np.abs(out[0][0]), 1.0)
    dg = np.linalg.norm(out[1][1] - out[0][1], axis=1) / np.linalg.norm(out[0][1], axis=1)
    parity.check("logp_rel", float(dlp.max()), "register vs generic BNN kernel")
    parity.check("grad_relnorm", float(dg.max()), "register vs generic BNN kernel")
    val = MLPEngine(c.spec, c.data["x_val"], c.data["y_val"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=C, device=cuda_device)
    preds = {}
    for fast in (1, 0):
        val.option("mlp_fast", fast)
        preds[fast] = val.forward(th)[1].double().cpu().numpy()
    parity.check("pred_elem", float(np.abs(preds[1] - preds[0]).max() / np.abs(preds[0]).max()),
                 "register vs generic BNN kernel, 300 validation rows (5 passes of 64)")
    res = {}
    for fast in (1, 0):
        eng.option("mlp_fast", fast)
        res[fast] = run_chains(EngineEvaluator(eng), th.clone(), 4, 30, 5e-4,
                               rng=ChainRNG(C, eng.K, cuda_device, seeds=[50 + i for i in range(C)]))
    assert torch.equal(res[1].accepted, res[0].accepted)
    n = int(res[1].counts.min())
    parity.check("pos_maxabs", float((res[1].samples[:, :n] - res[0].samples[:, :n]).abs().max()),
                 "register vs generic BNN trajectories, 4 x 30 steps")


def _accept_reference(lp, lp_new, ke0, ke1, logu):
    """HMCRunner.step's torch accept block."""
    d = (-lp + ke0) - (-lp_new + ke1)
    rho = torch.where(torch.isnan(d), torch.zeros_like(d), torch.clamp(d, max=0.0))
    ok = torch.isfinite(lp) & torch.isfinite(lp_new)
    return rho, ok, ok & (rho >= logu)


@pytest.mark.parametrize("burn", [0, 1])
@pytest.mark.parametrize("mass", [False, True])
def test_hmc_accept_kernel_matches_torch_block(burn, mass, cuda_device):
    """vihmc_hmc_accept (one launch per HMC iteration) == the torch accept block it replaces, bit for bit: rho
    (NaN for failed chains), the state selection after burn-in (in place + the sample row, a failed chain's row to
    the spare last row) and during burn-in (proposal / last returned / fallback), counts, accepted and trace."""
    import ctypes
    from vihmc import _lib
    torch.manual_seed(3)
    C, K, S, n = 7, 1000, 6, 2
    dev = cuda_device
    lp = -torch.rand(C, device=dev) * 10
    lp_new = lp + 0.05 * torch.randn(C, device=dev)
    lp_new[2] = float("nan")                            # a failed chain
    lp[5] = float("-inf")                               # another
    p0, p1 = torch.randn(C, K, device=dev), torch.randn(C, K, device=dev) * 1.001
    inv_mass = torch.rand(K, device=dev) + 0.5 if mass else None
    from vihmc.samplers import _kinetic
    ke0, ke1 = _kinetic(p0, inv_mass), _kinetic(p1, inv_mass)
    logu = torch.where(torch.arange(C, device=dev) % 2 == 0, torch.full((C,), -1e-3, device=dev),
                       torch.full((C,), -50.0, device=dev))
    rho_ref, ok, acc_ref = _accept_reference(lp, lp_new, ke0, ke1, logu)
    th1, g1 = torch.randn(C, K, device=dev), torch.randn(C, K, device=dev)
    last = [torch.randn(C, K, device=dev), lp.clone(), torch.randn(C, K, device=dev)]
    bp = [torch.randn(C, K, device=dev), torch.randn(C, device=dev), torch.randn(C, K, device=dev)]
    cur = [torch.empty(C, K, device=dev), torch.empty(C, device=dev), torch.empty(C, K, device=dev)]
    samples = torch.zeros(C, S, K, device=dev)
    counts = torch.ones(C, dtype=torch.long, device=dev)
    accepted = torch.zeros(C, 5, dtype=torch.bool, device=dev)
    trace = torch.zeros(C, 5, device=dev)
    rho, err = torch.empty(C, device=dev), torch.empty(C, dtype=torch.uint8, device=dev)
    exp_last = [t.clone() for t in last]
    exp_bp = [t.clone() for t in bp]

    def P(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None
    L = _lib.lib()
    _lib.check(L.vihmc_hmc_accept(C, K, n, burn, P(lp), P(lp_new), P(ke0), P(ke1), P(logu), P(th1), P(g1),
                                  P(last[0]), P(last[1]), P(last[2]), P(bp[0]), P(bp[1]), P(bp[2]), P(cur[0]),
                                  P(cur[1]), P(cur[2]), P(samples), S, P(counts), P(accepted), accepted.stride(0),
                                  P(trace), trace.stride(0), P(rho), P(err),
                                  ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "vihmc_hmc_accept")
    torch.cuda.synchronize()
    assert 0 < int(acc_ref.sum()) < C                    # both outcomes exercised
    assert torch.equal(accepted[:, n], acc_ref)
    assert torch.equal(err.bool(), ~ok)
    assert torch.equal(torch.isnan(rho), ~ok)
    assert torch.equal(rho[ok], rho_ref[ok])
    new = [th1, lp_new, g1]

    def sel(mask, a, b):
        return torch.where(mask[:, None] if a.dim() == 2 else mask, a, b)
    if not burn:
        nxt = [sel(acc_ref, nw, lr) for nw, lr in zip(new, exp_last)]
        for a, b in zip(last, nxt):
            assert torch.equal(a, b) or torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))
        row = torch.where(ok, torch.ones_like(counts), torch.full_like(counts, S - 1))
        for c in range(C):
            assert torch.equal(samples[c, int(row[c])], nxt[0][c])
        assert torch.equal(counts, 1 + ok.long())
        assert torch.equal(torch.nan_to_num(trace[:, n]), torch.nan_to_num(nxt[1]))
    else:
        fb = [sel(~ok, lr, b) for lr, b in zip(exp_last, exp_bp)]
        nxt = [sel(acc_ref, nw, f) for nw, f in zip(new, fb)]
        for a, b in zip(cur, nxt):
            assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))
        for a, b in zip(bp, [sel(acc_ref, nw, b) for nw, b in zip(new, exp_bp)]):
            assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))
        assert torch.equal(samples, torch.zeros_like(samples)) and torch.equal(counts, torch.ones_like(counts))
        assert torch.equal(torch.nan_to_num(trace[:, n]), torch.nan_to_num(nxt[1]))


@pytest.mark.parametrize("variant", ["hmc", "inv_mass", "nuts"])
def test_native_accept_equals_torch_accept(variant, cuda_device):
    """HMCRunner with the Metropolis step in one vihmc_hmc_accept launch == its torch form, on the engine: accept
    sequences, counts, samples, log-prob traces and (NUTS) adapted step sizes (burn-in and after)."""
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner, Sampler
    c = deeponet_case("deeponet_refshape")
    p = c.prob
    th0 = torch.tensor(c.thetas[0])
    C, S, L, eps = 3, 7, 3, 5e-3
    kw = dict(burn=2)
    if variant == "inv_mass":
        kw["inv_mass"] = torch.linspace(0.5, 1.5, th0.numel())
    if variant == "nuts":
        kw.update(sampler=Sampler.HMC_NUTS, burn=3)
    res = []
    for native in (True, False):
        eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                             c.prior_sd, c.loss, c.tau_out, max_chains=C, device=cuda_device)
        r = HMCRunner(EngineEvaluator(eng), th0[None].repeat(C, 1), S, L, eps,
                      rng=ChainRNG(C, th0.numel(), cuda_device, seeds=[40 + i for i in range(C)]), **kw)
        r._accept_native = native
        for _ in range(S):
            r.step()
        res.append(r.result())
        eng.close()
    a, b = res
    assert torch.equal(a.accepted, b.accepted)
    assert torch.equal(a.counts, b.counts)
    assert torch.equal(a.samples[:, :int(a.counts.max())], b.samples[:, :int(b.counts.max())])
    assert torch.equal(a.logp_trace, b.logp_trace)
    assert a.step_size == b.step_size


@pytest.mark.parametrize("C,K,mass", [(3, 1000, False), (2, 172401, True), (16, 17240, False)])
def test_kinetic_kernel(C, K, mass, cuda_device):
    """vihmc_kinetic (one launch) against an fp64 reference of hamiltorch's 0.5 p.p / 0.5 p.(inv_mass p): within one
    fp32 rounding of the exact value (fp64 sums of the fp32 products), and bitwise repeatable with the same workspace
    (its arrival counters reset themselves)."""
    import ctypes
    from vihmc import _lib
    L = _lib.lib()
    g = torch.Generator().manual_seed(5)
    p = torch.randn(C, K, generator=g).to(cuda_device)
    im = (torch.rand(K, generator=g) + 0.5).to(cuda_device) if mass else None
    S = int(L.vihmc_kinetic_slices(K))
    assert S >= 1
    part = torch.zeros(C * S, dtype=torch.float64, device=cuda_device)
    cnt = torch.zeros(C, dtype=torch.int32, device=cuda_device)

    def run():
        ke = torch.empty(C, device=cuda_device)
        P = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
        _lib.check(L.vihmc_kinetic(P(p), P(im), C, K, P(ke), P(part), P(cnt),
                                   ctypes.c_void_p(torch.cuda.current_stream(cuda_device).cuda_stream)), "vihmc_kinetic")
        torch.cuda.synchronize()
        return ke.cpu()
    a, b = run(), run()
    assert torch.equal(a, b)
    assert int(cnt.abs().sum()) == 0
    pc = p.cpu()
    q = pc * ((im.cpu() if mass else 1.0) * pc)                  # the fp32 products, as the kernel forms them
    ref = 0.5 * q.double().sum(1)
    assert torch.allclose(a.double(), ref, rtol=2 ** -23, atol=0)
    with pytest.raises(RuntimeError):
        _lib.check(L.vihmc_kinetic(None, None, C, K, None, None, None, None), "vihmc_kinetic")

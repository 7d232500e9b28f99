"""North-star parity at the bench workload's network shape and at full size, on the GPU.

* Sampler trajectories, accept sequences and the posterior-predictive mean of the batched HIP sampler
  (all bf16x6 MFMA forms on: the bench configuration) against the scalar hamiltorch restatement driving
  the reference's own torch log-prob (oracle/hamiltorch_ref.py + TorchDeepONetRef, fp32 CPU), on
  identical per-chain RNG streams:
    - ``deeponet_refshape``: width 100, depth 9, 101 branch inputs, K = 17,240 (reduced N = 8, P = 121),
      eps = 5e-3 so that about 1 in 5 proposals is rejected -- the accept decision is exercised;
    - ``deeponet_burgers``: the full Burgers shape (N = 1000, P = 10,201, K = 17,240), 1 chain x 5 samples
      x L = 7 at the reference's eps = 1e-4 (Operator_network/VI_HMC/main_VI_HMC_burgers.py:86-178,244-301).
* Config 4 (Operator_network/HMC/main_HMC_splitting.py:28-76,209-258,323-369) at the reference shape:
  D = 172,401 full-parameter closures over two shards of N/2 = 500 functions, with and without
  cfg.load_prior, against the reference-generated golden; two split-integrator samples against the oracle.

Tolerance statement. The Hamiltonians are fp32 sums of magnitude ~3e4, so rho = min(0, H0 - H1) is
resolved to ~4e-3 (one fp32 ulp of H is 2e-3) on both sides, and the engine's log-prob differs from the
CPU reference by fp32 rounding (< 1e-3 at |logp| = 2e4). An accept decision is therefore REQUIRED to agree
whenever the reference's margin |rho - log u| exceeds TAU_DECISION = 1e-2; a decision inside that band may
legitimately differ, and positions are compared up to the first such divergence. Positions: atol 1e-4
(max-abs). Posterior-predictive mean (north star): relative L2 < 1e-4.
"""
import numpy as np
import pytest
import torch

import parity
from goldens import deeponet_case, load, spec_of, split_burgers_case
from oracle import hamiltorch_ref as HR
from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout

pytestmark = pytest.mark.gpu

TAU_DECISION = 1e-2
POS_ATOL = 1e-4


def _layout(spec):
    return deeponet_layout(spec.in_branch, spec.width_branch, spec.depth_branch, spec.in_trunk, spec.width_trunk,
                           spec.depth_trunk, spec.out)


def _engine(c, C, dev):
    from vihmc.engine import DeepONetEngine, trunk_features
    p = c.prob
    return DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                          c.prior_sd, c.loss, c.tau_out, max_chains=C, device=dev)


def _trajectory_parity(res, ref_fn, th0, seeds, S, L, eps, burn=0, chains=None):
    """Compare chain chains[i] (default i) of the batched GPU run with the scalar reference sampler on seeds[i],
    started from th0 (one [K] start for every chain, or [C, K] with a start per chain of the run). Returns the
    aligned (gpu, ref) sample lists up to the first permitted divergence, and the smallest margin."""
    aligned = []
    min_margin = np.inf
    chains = list(range(len(seeds))) if chains is None else list(chains)
    for c, s in zip(chains, seeds):
        start = th0 if th0.dim() == 1 else th0[c]
        out, st = HR.sample(ref_fn, start.cpu(), S, L, eps, burn=burn, generator=torch.Generator().manual_seed(s),
                            return_stats=True)
        acc = res.accepted[c].cpu().tolist()
        margins = np.abs(np.asarray(st["rhos"]) - np.asarray(st["logus"]))
        min_margin = min(min_margin, float(margins.min()))
        n_ok = S
        for n in range(S):
            if acc[n] != st["accepts"][n]:
                assert margins[n] < TAU_DECISION, (c, n, acc[n], st["rhos"][n], st["logus"][n])
                n_ok = n
                break
        mine = [t.cpu() for t in res.chain(c)]
        # stored samples that precede iteration n_ok (1 initial + one per post-burn iteration)
        n_stored = 1 + max(0, n_ok - burn - 1) if n_ok < S else len(out)
        assert n_ok < S or len(mine) == len(out)
        dpos = max([float((a - b).abs().max()) for a, b in zip(mine[:n_stored], out[:n_stored])] + [0.0])
        parity.check("pos_maxabs", dpos, f"chain {c}, {n_stored} samples")
        aligned.append((mine[:n_stored], out[:n_stored], n_ok == S))
    return aligned, min_margin


def _predictive_mean_rel_l2(eng, ref, gpu_samples, ref_samples, dev):
    gpu = torch.stack(gpu_samples).to(dev)
    B = eng.max_chains
    preds = torch.cat([eng.forward(gpu[i:i + B])[1] for i in range(0, gpu.shape[0], B)])
    mean_gpu = preds.double().mean(0).cpu().numpy()
    mean_ref = np.mean([ref.forward(t.numpy())[1].astype(np.float64) for t in ref_samples], axis=0)
    return float(np.linalg.norm(mean_gpu - mean_ref) / np.linalg.norm(mean_ref))


def test_refshape_trajectories_accepts_and_predictive_mean(cuda_device):
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = deeponet_case("deeponet_refshape")
    seeds, S, L, eps, burn = [1000, 1001], 30, 7, 5e-3, 5
    eng = _engine(c, len(seeds), cuda_device)
    assert all(eng.get_option(k) == 1 for k in ("fwd_bf16x6", "contract_bf16x6", "bwd_bf16x6"))
    th0 = torch.tensor(c.thetas[0])
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(len(seeds), 1), S, L, eps, burn=burn,
                     rng=ChainRNG(len(seeds), th0.numel(), cuda_device, seeds=seeds))
    p = c.prob
    ref = TorchDeepONetRef(_layout(c.spec), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd,
                           c.loss, c.tau_out)
    aligned, min_margin = _trajectory_parity(res, ref.log_prob, th0, seeds, S, L, eps, burn)
    rate = float(res.accepted.float().mean())
    print(f"refshape: acceptance {rate:.2f}, smallest reference decision margin {min_margin:.2e}, "
          f"chains fully aligned: {[a[2] for a in aligned]}")
    assert 0.3 < rate < 0.99                      # the accept decision is exercised
    gpu_s = [t for a in aligned for t in a[0][1:]]
    ref_s = [t for a in aligned for t in a[1][1:]]
    rel = _predictive_mean_rel_l2(eng, ref, gpu_s, ref_s, cuda_device)
    print(f"refshape posterior-predictive mean over {len(gpu_s)} samples: rel L2 {rel:.2e}")
    parity.check("mean_rel_l2", rel, f"refshape, {len(gpu_s)} samples")


def test_burgers_full_shape_trajectory_and_predictive_mean(cuda_device):
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = deeponet_case("deeponet_burgers")
    seeds, S, L, eps = [1000], 5, 7, 1e-4
    eng = _engine(c, 1, cuda_device)
    th0 = torch.tensor(c.thetas[0])
    res = run_chains(EngineEvaluator(eng), th0[None], S, L, eps, rng=ChainRNG(1, th0.numel(), cuda_device, seeds=seeds))
    p = c.prob
    ref = TorchDeepONetRef(_layout(c.spec), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd,
                           c.loss, c.tau_out)
    aligned, min_margin = _trajectory_parity(res, ref.log_prob, th0, seeds, S, L, eps)
    print(f"burgers: smallest reference decision margin {min_margin:.2e}")
    assert aligned[0][2], "full-shape chain diverged from the reference sampler"
    rel = _predictive_mean_rel_l2(eng, ref, aligned[0][0][1:], aligned[0][1][1:], cuda_device)
    print(f"burgers posterior-predictive mean over {S} samples: rel L2 {rel:.2e}")
    parity.check("mean_rel_l2", rel, f"burgers, {S} samples")


# ------------------------------------------------------------------------------------------------
# Config 4: full-parameter split HMC at the reference shape
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def split_case():
    return split_burgers_case()


def _split_fns(case, load_prior, dev):
    from vihmc import configs
    from vihmc.operator import define_split_model_log_prob
    cfg = configs.load("burgers_hmc_splitting", load_prior=load_prior)
    p = case.prob
    tau_list = [torch.from_numpy(p.mu), torch.from_numpy(p.sigma)] if load_prior else [torch.tensor(cfg.prior_var)]
    shards = [tuple(torch.from_numpy(a) for a in sh) for sh in case.shards]
    return define_split_model_log_prob(case.spec, cfg.loss, shards, cfg.num_splits, tau_list, cfg.tau_out,
                                       device=dev, verbose=False, cfg=cfg)


@pytest.mark.parametrize("load_prior", [False, True])
def test_split_burgers_shard_closures_match_reference(split_case, load_prior, cuda_device):
    fns = _split_fns(split_case, load_prior, cuda_device)
    g = split_case.g
    sub = g["grad_subsample"]
    tag = "lp_" if load_prior else ""
    assert len(fns) == 2
    for m, f in enumerate(fns):
        eng = f._vihmc_engine
        assert eng.K == split_case.spec.n_params
        for t, th in enumerate(split_case.thetas):
            lp, gr = eng.logp_grad(torch.tensor(th, device=cuda_device)[None])
            ref = float(g[f"{tag}logp{t}_shard{m}"])
            note = f"load_prior={load_prior} shard {m} theta{t}"
            parity.check("logp_rel", abs(float(lp[0]) - ref) / max(abs(ref), 1.0), note)
            gr = gr[0].cpu().numpy().astype(np.float64)
            gs = np.asarray(g[f"{tag}grad{t}_shard{m}_sub"], np.float64)
            parity.check("grad_elem", np.abs(gr[sub] - gs).max() / np.abs(gs).max(), note)
            gn = float(g[f"{tag}grad{t}_shard{m}_norm"])
            parity.check("grad_norm_rel", abs(np.linalg.norm(gr) - gn) / gn, note)


def test_split_burgers_two_samples_vs_reference_sampler(split_case, cuda_device):
    from vihmc.samplers import Integrator, sample
    fns = _split_fns(split_case, False, cuda_device)
    th0 = torch.tensor(split_case.thetas[0], device=cuda_device)
    out = sample(fns, th0, num_samples=2, num_steps_per_sample=7, step_size=1e-4, integrator=Integrator.SPLITTING,
                 rng="per_chain", seed=5, verbose=True)
    lay = _layout(split_case.spec)
    refs = [TorchDeepONetRef(lay, x1, x2, y, None, np.arange(split_case.spec.n_params), 0.0, split_case.prior_sd,
                             split_case.loss, split_case.tau_out, prior_scale=2.0, full=True).log_prob
            for (x1, x2, y) in split_case.shards]
    ref, st = HR.sample(refs, th0.cpu(), 2, 7, 1e-4, integrator=HR.SPLITTING,
                        generator=torch.Generator().manual_seed(5), return_stats=True)
    margins = np.abs(np.asarray(st["rhos"]) - np.asarray(st["logus"]))
    print(f"split burgers: accepts {st['accepts']}, rho {st['rhos']}, margins {margins}")
    assert margins.min() > TAU_DECISION
    assert len(out) == len(ref)
    parity.check("pos_maxabs", max(float((a.cpu() - b).abs().max()) for a, b in zip(out, ref)), "2 split samples")


def test_split_loadprior_small_closures(cuda_device):
    """cfg.load_prior on the split path: D-length means/stds as the prior (main_HMC_splitting.py:341-345)."""
    from vihmc import configs
    from vihmc.operator import define_split_model_log_prob
    g = load("deeponet_split_loadprior")
    spec = spec_of(g)
    cfg = configs.load("burgers_hmc_splitting", load_prior=True, branch_depth=3, trunk_depth=3)
    shards = [(torch.from_numpy(g["branch_in"][4 * m:4 * m + 4]), torch.from_numpy(g["trunk_in"]),
               torch.from_numpy(g["y"][4 * m:4 * m + 4])) for m in range(2)]
    fns = define_split_model_log_prob(spec, "NLL", shards, 2, [torch.from_numpy(g["mu"]), torch.from_numpy(g["sigma"])],
                                      1.0, device=cuda_device, verbose=False, cfg=cfg)
    th = torch.tensor(g["theta"], device=cuda_device).requires_grad_()
    for m, f in enumerate(fns):
        lp = f(th)
        gr, = torch.autograd.grad(lp, th)
        ref = float(g[f"logp_shard{m}"])
        parity.check("logp_rel", abs(float(lp) - ref) / max(abs(ref), 1.0), f"shard {m}")
        gref = np.asarray(g[f"grad_shard{m}"], np.float64)
        parity.check("grad_relnorm", np.linalg.norm(gr.cpu().numpy() - gref) / np.linalg.norm(gref), f"shard {m}")

"""The splitting integrator's kicks and drifts inside the evaluations' gradient gathers (vihmc_split_step, used by
HMCRunner for Integrator.SPLITTING with two DeepONet shards, the reused end gradient and no mass matrix: config 4,
Operator_network/HMC/main_HMC_splitting.py:361-369) against the torch-op path of HMCRunner._trajectory
(engine attribute fused_split = False): samples, accepts, log-probs, momenta and gradients bit for bit -- every
update is one fma in both (torch.add(x, y, alpha=a) is fma(a, y, x) on the GPU, checked below).
"""
import numpy as np
import pytest
import torch

from goldens import split_burgers_case

pytestmark = pytest.mark.gpu


def test_torch_add_alpha_is_one_fma(cuda_device):
    """The premise: torch.add(alpha=) rounds once (fma), the form vihmc_split_step reproduces."""
    g = torch.Generator().manual_seed(0)
    p = torch.randn(1 << 16, generator=g)
    q = torch.randn(1 << 16, generator=g)
    h = 0.5 * 1.2345e-4
    t = torch.add(p.to(cuda_device), q.to(cuda_device), alpha=h).cpu().numpy()
    fma = (p.double().numpy() + np.float64(np.float32(h)) * q.double().numpy()).astype(np.float32)
    assert np.array_equal(t, fma)


def _engines(case, dev, C, fused, rows=None):
    from vihmc.engine import DeepONetEngine, trunk_features
    engs = []
    for (x1, x2, y) in case.shards:
        x1, y = np.asarray(x1), np.asarray(y)
        if rows is not None:
            x1, y = x1[:rows], y[:rows]
        e = DeepONetEngine(case.spec, x1, trunk_features(np.asarray(x2)), y, case.prob.mu,
                           np.arange(case.spec.n_params), 0.0, case.prior_sd, case.loss, case.tau_out, prior_scale=2.0,
                           max_chains=C, device=dev)
        e.fused_split = fused
        engs.append(e)
    return engs


@pytest.mark.parametrize("C,rows,S,L", [(1, None, 3, 7), (2, 64, 4, 5)])
def test_split_fused_trajectory_bitwise_equals_torch_updates(C, rows, S, L, cuda_device):
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner, Integrator
    case = split_burgers_case()
    th0 = torch.tensor(np.asarray(case.thetas[0], np.float32), device=cuda_device)[None].repeat(C, 1)
    res = []
    for fused in (True, False):
        engs = _engines(case, cuda_device, C, fused, rows)
        evs = [EngineEvaluator(e) for e in engs]
        r = HMCRunner(evs, th0, S, L, 1e-4, integrator=Integrator.SPLITTING,
                      rng=ChainRNG(C, th0.shape[1], cuda_device, seeds=[7 + i for i in range(C)]))
        assert r._fused_split(r._eps()) == fused
        for _ in range(S):
            r.step()
        res.append((r.samples.clone(), r.counts.clone(), r.accepted.clone(), r.trace.clone(),
                    [x.clone() for x in r.cur], [e.n_grad for e in evs], [e.n_value for e in evs]))
        for e in engs:
            e.close()
    a, b = res
    assert torch.equal(a[1], b[1])
    assert torch.equal(a[2], b[2])
    n = int(a[1].max())
    assert torch.equal(a[0][:, :n], b[0][:, :n])
    assert torch.equal(a[3], b[3])
    for x, y in zip(a[4], b[4]):
        assert torch.equal(x, y)
    assert a[5] == b[5] and a[6] == b[6]          # the same evaluation counts
    assert bool(a[2].any())                       # the chains move


def test_split_step_api_contract(cuda_device):
    """vihmc_split_step's argument checks: mode, in-place operands, the scatter target's layout."""
    case = split_burgers_case()
    e0, e1 = _engines(case, cuda_device, 1, True, rows=32)
    th = torch.tensor(np.asarray(case.thetas[0], np.float32), device=cuda_device)[None].contiguous()
    p = torch.zeros_like(th)
    with pytest.raises(RuntimeError):
        e0.split_step(th, p, 3, 1e-4)
    with pytest.raises(ValueError):
        e0.split_step(th.double(), p, 1, 1e-4)
    lp, g = e0.split_step(th.clone(), p.clone(), 2, 1e-4, want_logp=True)
    lp_ref, g_ref = e0.logp_grad(th)
    assert torch.equal(g, g_ref) and torch.equal(lp, lp_ref)
    e0.close()
    e1.close()

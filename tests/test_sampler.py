"""Batched sampler (vihmc.samplers) vs the scalar hamiltorch restatement (oracle/hamiltorch_ref.py).

Sampler parity is unpinned (hamiltorch is absent); these tests pin the batched,
device-style implementation to the scalar restatement on identical RNG streams, on the CPU through
the autograd evaluator with the oracle's torch BNN log-prob (the same function the reference runs).
Trajectories are bit-identical except for the kinetic-energy summation order, so accept decisions
must agree exactly and samples to fp32 rounding.
"""
import numpy as np
import pytest
import torch

from goldens import bnn_case
from oracle import hamiltorch_ref as HR
from oracle.bnn_ref import TorchBNNRef, mlp_layout
from vihmc import samplers as S


def bnn_fn(x=None, y=None, name="bnn_vi_hmc", prior_scale=1.0):
    c = bnn_case(name)
    g = c.g
    x = c.data["x_train"] if x is None else x
    y = c.data["y_train"] if y is None else y
    ref = TorchBNNRef(mlp_layout(), x, y, g["mu"], c.idx, prior_list=list(g["prior_var"]), loss=c.loss,
                      tau_out=c.tau_out, prior_scale=prior_scale)
    return ref.log_prob, torch.tensor(c.thetas[0]), c


def run_both(fn, th0, seeds, strict_rng=False, **kw):
    C = len(seeds)
    K = th0.shape[0]
    ev = S.AutogradEvaluator(fn, K, "cpu") if not isinstance(fn, list) else [S.AutogradEvaluator(f, K, "cpu") for f in fn]
    rng = S.ChainRNG(C, K, "cpu", seeds=seeds)
    res = S.run_chains(ev, th0[None].repeat(C, 1), rng=rng, strict_rng=strict_rng, **kw)
    refs = []
    for s in seeds:
        g = torch.Generator().manual_seed(s)
        sampler = HR.HMC_NUTS if kw.get("sampler") == S.Sampler.HMC_NUTS else HR.HMC
        integ = HR.SPLITTING if kw.get("integrator") == S.Integrator.SPLITTING else HR.IMPLICIT
        out, st = HR.sample(fn, th0, kw["num_samples"], kw["num_steps_per_sample"], kw["step_size"],
                            burn=kw.get("burn", 0), sampler=sampler, integrator=integ, generator=g,
                            inv_mass=kw.get("inv_mass"), return_stats=True)
        refs.append((out, st))
    return res, refs


def check(res, refs, atol=1e-5):
    for c, (out, st) in enumerate(refs):
        assert res.accepted[c].tolist() == st["accepts"]
        mine = res.chain(c)
        assert len(mine) == len(out)
        for a, b in zip(mine, out):
            torch.testing.assert_close(a, b, rtol=0, atol=atol)


def test_rng_stream_matches_hamiltorch_call_order():
    K = 37
    rng = S.ChainRNG(2, K, "cpu", seeds=[5, 9])
    z, lu = rng.draw()
    assert z.shape == (2, K)
    for c, s in enumerate([5, 9]):
        g = torch.Generator().manual_seed(s)
        zr = HR.gibbs(torch.zeros(K), None, g)
        ur = torch.log(torch.rand(1, generator=g))
        assert torch.equal(z[c], zr) and lu[c] == ur[0]


def test_single_chain_matches_scalar_hamiltorch():
    fn, th0, _ = bnn_fn()
    res, refs = run_both(fn, th0, [3], num_samples=12, num_steps_per_sample=8, step_size=5e-4)
    check(res, refs)
    assert 0 < int(res.accepted.sum()) <= 12


def test_multi_chain_each_chain_is_its_seeded_scalar_run():
    fn, th0, _ = bnn_fn()
    res, refs = run_both(fn, th0, [0, 1, 2], num_samples=8, num_steps_per_sample=6, step_size=5e-4)
    check(res, refs)


def test_burn_bookkeeping_and_rejections():
    """Large step -> frequent rejections; burn > 0 exercises param_burn_prev and the post-burn revert to
    ret_params[-1] (hamiltorch keeps the *initial* params there until the first post-burn accept)."""
    fn, th0, _ = bnn_fn()
    res, refs = run_both(fn, th0, [7, 8], num_samples=14, num_steps_per_sample=5, step_size=3e-3, burn=4)
    check(res, refs)
    assert (~res.accepted).any(), "test needs some rejections"
    assert int(res.counts[0]) == len(refs[0][0]) == 1 + 14 - 1 - 4


def test_reuse_endpoint_grad_is_exact():
    fn, th0, _ = bnn_fn()
    kw = dict(num_samples=6, num_steps_per_sample=4, step_size=1e-3)
    a = S.run_chains(S.AutogradEvaluator(fn, th0.numel(), "cpu"), th0[None], rng=S.ChainRNG(1, th0.numel(), "cpu", [4]),
                     reuse_endpoint_grad=True, **kw)
    b = S.run_chains(S.AutogradEvaluator(fn, th0.numel(), "cpu"), th0[None], rng=S.ChainRNG(1, th0.numel(), "cpu", [4]),
                     reuse_endpoint_grad=False, **kw)
    assert torch.equal(a.samples[:, :int(a.counts[0])], b.samples[:, :int(b.counts[0])])
    assert a.n_grad_evals == 1 + 6 * 4 and b.n_grad_evals == 1 + 6 * 5


def test_nuts_dual_averaging_matches():
    fn, th0, _ = bnn_fn()
    res, refs = run_both(fn, th0, [11, 12], num_samples=10, num_steps_per_sample=5, step_size=2e-3, burn=5,
                         sampler=S.Sampler.HMC_NUTS)
    check(res, refs, atol=1e-5)
    for c, (_, st) in enumerate(refs):
        assert res.step_size[c] == pytest.approx(st["step_sizes"][-1], rel=0, abs=0)


def test_diagonal_inverse_mass():
    fn, th0, _ = bnn_fn()
    inv_mass = torch.linspace(0.5, 2.0, th0.numel())
    res, refs = run_both(fn, th0, [21], num_samples=6, num_steps_per_sample=5, step_size=5e-4, inv_mass=inv_mass)
    check(res, refs)


def test_splitting_integrator_matches():
    c = bnn_case("bnn_vi_hmc")
    x, y = c.data["x_train"], c.data["y_train"]
    fns = [bnn_fn(x[:10], y[:10], prior_scale=2.0)[0], bnn_fn(x[10:], y[10:], prior_scale=2.0)[0]]
    th0 = torch.tensor(c.thetas[0])
    res, refs = run_both(fns, th0, [31, 32], num_samples=6, num_steps_per_sample=4, step_size=5e-4,
                         integrator=S.Integrator.SPLITTING)
    check(res, refs)
    # 2 new gradient evaluations per step after the first (turnaround + step boundary reuse)
    assert res.n_grad_evals == 2 * (1 + 6 * 4 * 2)


def test_logprob_error_is_rejection_without_storage():
    """A log-prob that is NaN beyond a threshold: hamiltorch raises LogProbError -> reject, params revert
    to ret_params[-1], nothing appended."""
    base, th0, _ = bnn_fn()
    thr = float(th0[0]) + 2e-3

    def fn(p):
        lp = base(p)
        return torch.where(p[0] > thr, torch.full_like(lp, float("nan")), lp)

    res, refs = run_both(fn, th0, [41, 42, 43], num_samples=12, num_steps_per_sample=6, step_size=2e-3, burn=2,
                         strict_rng=True)
    check(res, refs)
    assert any(len(o) < 1 + 12 - 1 - 2 for o, _ in refs), "test needs at least one LogProbError"


def test_sample_entry_point_generic_closure():
    fn, th0, _ = bnn_fn()
    torch.manual_seed(0)
    out = S.sample(fn, th0, num_samples=5, num_steps_per_sample=3, step_size=5e-4, verbose=True)
    torch.manual_seed(0)
    ref = HR.sample(fn, th0, 5, 3, 5e-4)
    assert len(out) == len(ref)
    for a, b in zip(out, ref):
        torch.testing.assert_close(a, b, rtol=0, atol=1e-5)


def test_sample_entry_point_global_rng_skips_draw_on_logprob_error():
    """hamiltorch's drop-in (rng='global'): after a LogProbError no accept uniform is drawn, so the global
    CPU stream -- and every later momentum and accept draw -- stays aligned with hamiltorch's."""
    base, th0, _ = bnn_fn()
    thr = float(th0[0]) + 2e-3

    def fn(p):
        lp = base(p)
        return torch.where(p[0] > thr, torch.full_like(lp, float("nan")), lp)

    torch.manual_seed(3)
    out = S.sample(fn, th0, num_samples=14, num_steps_per_sample=6, step_size=2e-3, burn=2, verbose=True)
    torch.manual_seed(3)
    ref, st = HR.sample(fn, th0, 14, 6, 2e-3, burn=2, return_stats=True)
    assert any(r != r for r in st["rhos"]), "test needs at least one LogProbError"
    assert len(out) == len(ref)
    for a, b in zip(out, ref):
        torch.testing.assert_close(a, b, rtol=0, atol=1e-5)

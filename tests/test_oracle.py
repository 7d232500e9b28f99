"""The oracle is pinned before it is trusted: both CPU restatements vs the reference-generated goldens.

Tolerances: the torch restatement runs the reference's own ops in fp32 -> logp to 1e-6 relative,
gradient to 1e-5 of its norm. The numpy restatement is fp64 and differs from the fp32 reference
by the reference's own rounding -> logp 2e-5 relative (+1e-3 absolute), gradient 1e-4 of its norm.
"""
import numpy as np
import pytest

from goldens import BNN_CASES, DEEPONET_CASES, bnn_case, deeponet_case, load, spec_of, split_burgers_case
from oracle.bnn_ref import TorchBNNRef, mlp_layout, np_bnn_logp_grad
from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout, np_logp_grad


def layout_of(spec):
    return deeponet_layout(spec.in_branch, spec.width_branch, spec.depth_branch, spec.in_trunk, spec.width_trunk,
                           spec.depth_trunk, spec.out)


def rel_norm(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def test_layout_matches_reference_offsets():
    br, tr, D = deeponet_layout()
    assert D == 172401
    assert br[0].w_off == 1 and br[0].b_off == 10101 and br[-1].b_off == 90901
    assert tr[0].w_off == 91001 and tr[0].b_off == 91501 and tr[-1].b_off + 100 == 172401
    layers, Dn = mlp_layout()
    assert Dn == 141 and [(l.w_off, l.b_off) for l in layers] == [(0, 10), (20, 120), (130, 140)]


@pytest.mark.parametrize("name", DEEPONET_CASES)
def test_deeponet_torch_oracle_matches_golden(name):
    c = deeponet_case(name)
    p = c.prob
    ref = TorchDeepONetRef(layout_of(c.spec), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd,
                           c.loss, c.tau_out, full=c.full)
    for t, th in enumerate(c.thetas):
        lp, g = ref.logp_grad(th)
        assert lp == pytest.approx(float(c.g[f"logp{t}"]), rel=1e-6, abs=1e-4)
        if f"grad{t}" in c.g:
            assert rel_norm(g, c.g[f"grad{t}"]) < 1e-5
        else:
            sub = c.g["grad_subsample"]
            np.testing.assert_allclose(g[sub], c.g[f"grad{t}_sub"], rtol=1e-4, atol=1e-5 * np.abs(g).max())
            assert np.linalg.norm(g.astype(np.float64)) == pytest.approx(float(c.g[f"grad{t}_norm"]), rel=1e-5)
        if f"pred{t}" in c.g:
            _, out = ref.forward(th)
            np.testing.assert_allclose(out, c.g[f"pred{t}"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", DEEPONET_CASES)
def test_deeponet_numpy_oracle_matches_golden(name):
    c = deeponet_case(name)
    p = c.prob
    for t, th in enumerate(c.thetas):
        lp, g, out = np_logp_grad(layout_of(c.spec), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, th, c.prior_mu,
                                  c.prior_sd, c.loss, c.tau_out, full=c.full)
        gl = float(c.g[f"logp{t}"])
        assert lp == pytest.approx(gl, rel=2e-5, abs=1e-3)
        if f"grad{t}" in c.g:
            assert rel_norm(g, c.g[f"grad{t}"]) < 1e-4
        else:
            sub = c.g["grad_subsample"]
            gs = c.g[f"grad{t}_sub"]
            np.testing.assert_allclose(g[sub], gs, rtol=1e-3, atol=1e-4 * np.abs(gs).max())
        if f"pred{t}" in c.g:
            np.testing.assert_allclose(out, c.g[f"pred{t}"], rtol=1e-5, atol=1e-5)


@pytest.mark.slow
def test_deeponet_full_burgers_shape_golden():
    """N=1000, P=10201, K=17240 -- the bench workload itself, pinned against the reference."""
    c = deeponet_case("deeponet_burgers")
    p = c.prob
    lp, g, _ = np_logp_grad(layout_of(c.spec), p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, c.thetas[0],
                            c.prior_mu, c.prior_sd, c.loss, c.tau_out)
    assert lp == pytest.approx(float(c.g["logp0"]), rel=2e-5, abs=1e-2)
    sub = c.g["grad_subsample"]
    np.testing.assert_allclose(g[sub], c.g["grad0_sub"], rtol=2e-3, atol=2e-4 * np.abs(c.g["grad0_sub"]).max())
    assert np.linalg.norm(g) == pytest.approx(float(c.g["grad0_norm"]), rel=1e-4)


def test_deeponet_split_shards_golden():
    """Full-parameter split closures: each shard = N/2 rows, prior divided by num_splits=2."""
    g = load("deeponet_split")
    spec = spec_of(g)
    lay = layout_of(spec)
    for m in range(2):
        sl = slice(4 * m, 4 * (m + 1))
        idx = np.arange(spec.n_params)
        lp, gr, _ = np_logp_grad(lay, g["branch_in"][sl], g["trunk_in"], g["y"][sl], None, idx, g["theta"], 0.0,
                                 float(np.sqrt(g["prior_var"])), str(g["loss"]), float(g["tau_out"]), prior_scale=2.0,
                                 full=True)
        assert lp == pytest.approx(float(g[f"logp_shard{m}"]), rel=2e-5, abs=1e-3)
        assert rel_norm(gr, g[f"grad_shard{m}"]) < 1e-4


def test_deeponet_split_loadprior_golden():
    """Split closures with cfg.load_prior: prior Normal(means[D], stds[D]) / num_splits per shard
    (Operator_network/HMC/main_HMC_splitting.py:122-129,341-345)."""
    g = load("deeponet_split_loadprior")
    spec = spec_of(g)
    lay = layout_of(spec)
    idx = np.arange(spec.n_params)
    for m in range(2):
        sl = slice(4 * m, 4 * (m + 1))
        lp, gr, _ = np_logp_grad(lay, g["branch_in"][sl], g["trunk_in"], g["y"][sl], None, idx, g["theta"], g["mu"],
                                 g["sigma"], str(g["loss"]), float(g["tau_out"]), prior_scale=2.0, full=True)
        assert lp == pytest.approx(float(g[f"logp_shard{m}"]), rel=2e-5, abs=1e-3)
        assert rel_norm(gr, g[f"grad_shard{m}"]) < 1e-4


@pytest.mark.parametrize("load_prior", [False, True])
def test_deeponet_split_burgers_golden(load_prior):
    """Config 4 at the reference shape: D = 172,401, two shards of N/2 = 500 functions x P = 10,201 points
    (the torch restatement: fp32, the reference's ops)."""
    c = split_burgers_case()
    g, p = c.g, c.prob
    lay = layout_of(c.spec)
    pm, ps = (p.mu, p.sigma) if load_prior else (0.0, c.prior_sd)
    tag = "lp_" if load_prior else ""
    sub = g["grad_subsample"]
    for m, (x1, x2, y) in enumerate(c.shards):
        ref = TorchDeepONetRef(lay, x1, x2, y, None, np.arange(c.spec.n_params), pm, ps, c.loss, c.tau_out,
                               prior_scale=2.0, full=True)
        for t, th in enumerate(c.thetas):
            lp, gr = ref.logp_grad(th)
            assert lp == pytest.approx(float(g[f"{tag}logp{t}_shard{m}"]), rel=1e-6)
            gs = g[f"{tag}grad{t}_shard{m}_sub"]
            np.testing.assert_allclose(gr[sub], gs, rtol=1e-4, atol=1e-5 * np.abs(gs).max())
            assert np.linalg.norm(gr.astype(np.float64)) == pytest.approx(float(g[f"{tag}grad{t}_shard{m}_norm"]),
                                                                          rel=1e-5)


def test_deeponet_nuts_closure_golden():
    """NUTS_DeepOnets.py closure: full parameters, prior of tensor i = Normal(0, tau_i * 0.5) (reference quirk)."""
    from vihmc.engine import prior_per_tensor
    g = load("deeponet_nuts")
    spec = spec_of(g)
    D = spec.n_params
    ps = prior_per_tensor(list(g["sizes"]), D, list(0.5 * g["taus"].astype(np.float64)))
    lp, gr, _ = np_logp_grad(layout_of(spec), g["branch_in"], g["trunk_in"], g["y"], None, np.arange(D), g["theta"], 0.0,
                             ps, str(g["loss"]), float(g["tau_out"]), full=True)
    assert lp == pytest.approx(float(g["logp"]), rel=2e-5, abs=1e-3)
    assert rel_norm(gr, g["grad"]) < 1e-4


def test_deeponet_sample_data_golden():
    """cfg.sample_data (main_VI_HMC_burgers.py:127-137): three successive reference calls after random.seed(seed),
    each at random.sample(range(P_all), p) trunk rows -- the stored rows replay from the seed, and the oracle at
    those rows gives the reference's outputs."""
    import random
    g = load("deeponet_sampledata")
    spec = spec_of(g)
    P_all, p = g["trunk_in"].shape[1], int(g["p"])
    random.seed(int(g["seed"]))
    for t in range(3):
        ind = np.asarray(random.sample(range(P_all), p))
        np.testing.assert_array_equal(ind, g[f"ind{t}"])
        lp, gr, _ = np_logp_grad(layout_of(spec), g["branch_in"], g["trunk_in"][:, ind], g["y"][:, ind], g["mu"],
                                 g["grad_ind"], g[f"theta{t}"], 0.0, float(np.sqrt(g["prior_var"])), str(g["loss"]),
                                 float(g["tau_out"]))
        assert lp == pytest.approx(float(g[f"logp{t}"]), rel=2e-5, abs=1e-3)
        assert rel_norm(gr, g[f"grad{t}"]) < 1e-4
    assert abs(float(g["logp0"]) - float(g["logp2"])) > 1e-3     # same theta, different rows


@pytest.mark.parametrize("name", BNN_CASES)
def test_bnn_oracles_match_golden(name):
    c = bnn_case(name)
    g = c.g
    lay = mlp_layout()
    load_prior = (g["mu"][c.idx], g["sd"][c.idx]) if bool(g["load_prior"]) else None
    tref = TorchBNNRef(lay, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, prior_list=list(g["prior_var"]),
                       loss=c.loss, tau_out=c.tau_out, load_prior=load_prior)
    for t, th in enumerate(c.thetas):
        lp, gr = tref.logp_grad(th)
        assert lp == pytest.approx(float(g[f"logp{t}"]), rel=1e-6)
        assert rel_norm(gr, g[f"grad{t}"]) < 1e-5
        lpn, grn, _ = np_bnn_logp_grad(lay, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, th, c.prior_mu,
                                       c.prior_sd, c.loss, c.tau_out)
        assert lpn == pytest.approx(float(g[f"logp{t}"]), rel=2e-5)
        assert rel_norm(grn, g[f"grad{t}"]) < 1e-4
        # predict_model path on the validation set
        lpv, _, pred = np_bnn_logp_grad(lay, c.data["x_val"], c.data["y_val"], g["mu"], c.idx, th, c.prior_mu,
                                        c.prior_sd, c.loss, c.tau_out)
        assert lpv == pytest.approx(float(g[f"val_logp{t}"]), rel=2e-5)
        np.testing.assert_allclose(pred, g[f"val_pred{t}"], rtol=1e-5, atol=1e-5)

"""CPU checks of the reference-compatible surface (no kernel calls)."""
import numpy as np
import pytest
import torch

from goldens import load


def test_deeponet_module_init_matches_reference():
    from vihmc.operator import DeepONet, flatten
    torch.manual_seed(123)
    net = DeepONet(16, 16, 12, 5, 3, 3, "tanh", None)
    ref = load("init_fixtures")["deeponet_16_12_3"]
    np.testing.assert_array_equal(flatten(net).detach().numpy(), ref)
    assert net.spec.n_params == ref.size


def test_bnn_get_model_init_matches_reference():
    from vihmc import configs
    from vihmc.bnn import flatten, get_model, spec_of
    torch.manual_seed(123)
    net = get_model(configs.load("nn_vi_hmc"), True)
    ref = load("init_fixtures")["bnn_10_10"]
    np.testing.assert_array_equal(flatten(net).detach().numpy(), ref)
    s = spec_of(net)
    assert s.n_params == 141 and s.width == (10, 10) and s.act == "tanh"


def test_unflatten_views_follow_named_parameters():
    from vihmc.operator import DeepONet, flatten, unflatten
    net = DeepONet(16, 16, 12, 5, 3, 3, "tanh", None)
    flat = flatten(net).detach()
    views = unflatten(net, flat)
    for v, p in zip(views, net.parameters()):
        assert torch.equal(v, p.detach())
    lay = net.spec
    assert views[1].data_ptr() == flat[lay.branch[0].w_off:].data_ptr()


def test_forward_matches_oracle_functional_model():
    from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout
    from vihmc.data import deeponet_problem
    from vihmc.layout import DeepONetSpec
    from vihmc.operator import DeepONet, flatten
    torch.manual_seed(0)
    net = DeepONet(16, 16, 12, 5, 3, 3, "tanh", None)
    spec = DeepONetSpec(16, 16, 12, 5, 3, 3)
    p = deeponet_problem(seed=1, n=4, nt=3, nx=5, spec=spec, k=None)
    flat = flatten(net).detach().numpy()
    ref = TorchDeepONetRef(deeponet_layout(12, 16, 3, 5, 16, 3), p.branch_in, p.trunk_in, p.y, flat,
                           np.arange(flat.size), full=True)
    with torch.no_grad():
        out = net(torch.from_numpy(p.branch_in), torch.from_numpy(p.trunk_in))
        exp = ref.functional_model(torch.from_numpy(flat)).squeeze(1)
    torch.testing.assert_close(out, exp)


def test_l2_relative_error():
    from vihmc.operator import l2_relative_error
    y = np.array([[3.0, 4.0], [1.0, 0.0]])
    e = l2_relative_error(y, y * 1.5)
    np.testing.assert_allclose(e, [0.5, 0.5])
    with pytest.raises(ValueError):
        l2_relative_error(y, y[:1])


def test_synthetic_burgers_data_shapes():
    from vihmc import configs
    from vihmc.operator import get_burgers_data
    cfg = configs.load("burgers_vi_hmc", N_train=6, N_valid=2)
    tr, va = get_burgers_data(cfg, mat_path="/nonexistent.mat")
    assert tr[0].shape == (6, 1, 101) and tr[1].shape == (1, 10201, 2) and tr[2].shape == (6, 10201)
    assert va[0].shape == (2, 1, 101) and va[2].shape == (2, 10201)


def test_artefact_roundtrip(tmp_path):
    from vihmc.data import load_vi_artefacts, save_vi_artefacts
    mu = np.arange(10, dtype=np.float32)
    sd = mu + 1
    idx = np.array([1, 5, 7])
    save_vi_artefacts(str(tmp_path), "u1", mu, sd, idx)
    m, s, i = load_vi_artefacts(str(tmp_path), "u1")
    assert np.array_equal(m, mu) and np.array_equal(s, sd) and np.array_equal(i, idx)


def test_ess_iid_and_correlated():
    from vihmc.diagnostics import ess
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 4000, generator=g, dtype=torch.float64)
    e = ess(x)
    assert torch.all((e > 2800) & (e < 5200))
    ar = torch.zeros(4, 4000, dtype=torch.float64)
    for t in range(1, 4000):
        ar[:, t] = 0.9 * ar[:, t - 1] + x[:, t]
    e2 = ess(ar)                                    # tau = (1+0.9)/(1-0.9) = 19
    assert torch.all((e2 > 4000 / 19 * 0.6) & (e2 < 4000 / 19 * 1.6))

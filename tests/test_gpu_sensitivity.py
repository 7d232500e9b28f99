"""Sensitivity step on the GPU (vihmc_sensitivity, vihmc_sens.hip) against the reference's own
eval_std_dydw outputs (tests/golden/sens_*.npz) and the fp64 oracle (oracle/sensitivity_ref.py); at the
Burgers shapes (N=1000, P=10201, p=100 points per function) through size-independent properties and an
oracle check on a subset of functions."""
import time

import numpy as np
import pytest
import torch

from oracle.deeponet_ref import deeponet_layout
from oracle.sensitivity_ref import np_sensitivity_deeponet
from sens_cases import SENS_BNN, SENS_DEEPONET, assert_scores_close, bnn_sens_case, deeponet_sens_case

pytestmark = pytest.mark.gpu


def _batches(g):
    return [(torch.from_numpy(g["branch_in"][i]).view(1, 1, -1),
             torch.from_numpy(g["trunk_in"][g["pts"][i]]).view(1, -1, 2)) for i in range(g["pts"].shape[0])]


@pytest.mark.parametrize("name", SENS_DEEPONET)
def test_deeponet_scores_match_reference(name, cuda_device):
    from vihmc.sensitivity import eval_std_dydw, sensitivity_scores
    c = deeponet_sens_case(name)
    g = c.g
    s = eval_std_dydw(_batches(g), c.spec, g["mu"], g["sd"], device=cuda_device)
    assert s.dtype == np.float32 and s.shape == g["scores"].shape
    assert_scores_close(s, g["scores"])
    s2 = sensitivity_scores(c.spec, g["branch_in"], g["trunk_in"], g["pts"], g["mu"], g["sd"], device=cuda_device)
    assert_scores_close(s2, np_sensitivity_deeponet(c.layout, g["mu"], g["sd"], g["branch_in"], g["trunk_in"],
                                                    g["pts"], c.act))


@pytest.mark.parametrize("name", SENS_BNN)
def test_bnn_scores_match_reference(name, cuda_device):
    from vihmc.layout import MLPSpec
    from vihmc.sensitivity import eval_std_dydw
    c = bnn_sens_case(name)
    spec = MLPSpec(width=c.width, act=c.act)
    s = eval_std_dydw((torch.from_numpy(c.g["x_val"]), None), spec, c.g["mu"], c.g["sd"], device=cuda_device)
    assert_scores_close(s, c.g["scores"])


def test_batches_of_two_weigh_like_the_reference(cuda_device):
    """DataLoader(batch_size=2): per-batch means averaged over batches -- equal sizes = mean over pairs."""
    from vihmc.sensitivity import eval_std_dydw
    c = deeponet_sens_case("sens_deeponet_small")
    g = c.g
    b1 = _batches(g)
    b2 = [(torch.cat([b1[i][0], b1[i + 1][0]]), torch.cat([b1[i][1], b1[i + 1][1]])) for i in range(0, len(b1), 2)]
    assert_scores_close(eval_std_dydw(b2, c.spec, g["mu"], g["sd"], device=cuda_device), g["scores"])


def test_burgers_shape_properties(cuda_device):
    from vihmc.data import deeponet_problem
    from vihmc.layout import DeepONetSpec
    from vihmc.sensitivity import sample_points, sensitivity_scores
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    pts = sample_points(prob.N, prob.P, 100, seed=5)
    mu, sd = prob.mu, prob.sigma
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s = sensitivity_scores(spec, prob.branch_in, prob.trunk_in, pts, mu, sd, device=cuda_device)
    dt = time.perf_counter() - t0
    print(f"Burgers sensitivity (N=1000, P=10201, p=100, D={spec.n_params}): {dt * 1e3:.1f} ms incl. plan setup")
    assert np.isfinite(s).all() and (s >= 0).all()
    assert s[0] == pytest.approx(float(sd[0]) ** 2, rel=1e-6)
    # bitwise deterministic
    assert np.array_equal(s, sensitivity_scores(spec, prob.branch_in, prob.trunk_in, pts, mu, sd, device=cuda_device))
    # sigma enters as sigma^2 elementwise
    raw = sensitivity_scores(spec, prob.branch_in, prob.trunk_in, pts, mu, None, device=cuda_device)
    np.testing.assert_allclose(s, raw * sd.astype(np.float64) ** 2, rtol=1e-5, atol=0)
    # the pair mean splits: points 0..49 and 50..99 of every function
    h1 = sensitivity_scores(spec, prob.branch_in, prob.trunk_in, pts[:, :50], mu, None, device=cuda_device)
    h2 = sensitivity_scores(spec, prob.branch_in, prob.trunk_in, pts[:, 50:], mu, None, device=cuda_device)
    np.testing.assert_allclose(0.5 * (h1.astype(np.float64) + h2), raw, rtol=2e-5, atol=1e-6 * raw.max())
    # oracle on a subset of functions at full width / depth / P
    lay = deeponet_layout()
    sub = np.array([3, 517])
    so = sensitivity_scores(spec, prob.branch_in[sub], prob.trunk_in, pts[sub], mu, sd, device=cuda_device)
    ref = np_sensitivity_deeponet(lay, mu, sd, prob.branch_in[sub], prob.trunk_in, pts[sub])
    assert_scores_close(so, ref)


def test_full_grid_points(cuda_device):
    """Every function on many shared points (trunk groups with hundreds of seeds, several tasks each)."""
    from vihmc.data import deeponet_problem
    from vihmc.layout import DeepONetSpec
    from vihmc.sensitivity import sensitivity_scores
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    sub = np.arange(0, 1000, 100)
    pts = np.tile(np.arange(0, prob.P, 7, dtype=np.int32)[:300], (sub.size, 1))
    s = sensitivity_scores(spec, prob.branch_in[sub], prob.trunk_in, pts, prob.mu, prob.sigma, device=cuda_device)
    ref = np_sensitivity_deeponet(deeponet_layout(), prob.mu, prob.sigma, prob.branch_in[sub], prob.trunk_in, pts)
    assert_scores_close(s, ref)

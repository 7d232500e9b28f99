"""CPU checks of the sensitivity step: the numpy oracle (oracle/sensitivity_ref.py) against the scores the
reference's own eval_std_dydw produced (tests/golden/sens_*.npz), and the host-side logic of
vihmc.sensitivity (batch grouping, point dedup, captured_var / index selection)."""
import numpy as np
import pytest

from oracle.sensitivity_ref import captured_var as ref_captured_var
from oracle.sensitivity_ref import np_sensitivity_deeponet, np_sensitivity_mlp, select_indices as ref_select
from sens_cases import SENS_BNN, SENS_DEEPONET, assert_scores_close, bnn_sens_case, deeponet_sens_case


@pytest.mark.parametrize("name", SENS_DEEPONET)
def test_oracle_deeponet_matches_reference(name):
    c = deeponet_sens_case(name)
    g = c.g
    s = np_sensitivity_deeponet(c.layout, g["mu"], g["sd"], g["branch_in"], g["trunk_in"], g["pts"], c.act)
    assert_scores_close(s, g["scores"])
    assert s[0] == pytest.approx(float(g["sd"][0]) ** 2, rel=1e-6)      # d f / d b = 1


@pytest.mark.parametrize("name", SENS_BNN)
def test_oracle_bnn_matches_reference(name):
    c = bnn_sens_case(name)
    s = np_sensitivity_mlp(c.layers, c.g["mu"], c.g["sd"], c.g["x_val"], c.act)
    assert_scores_close(s, c.g["scores"])


def test_captured_var_and_selection():
    from vihmc.sensitivity import captured_var, select_indices
    imp = deeponet_sens_case("sens_deeponet_w100").g["scores"]
    for thr in (0.5, 0.9, 0.99):
        n = captured_var(imp, thr)
        assert n == ref_captured_var(imp, thr)
        ind = select_indices(imp, thr)
        assert np.array_equal(ind, ref_select(imp, thr))
        assert ind.size == n and np.all(np.diff(ind) > 0)
        # the selected scores are the n largest
        assert np.min(imp[ind]) >= np.sort(imp)[::-1][n - 1]


def test_operator_batches_group_and_dedup():
    import torch
    from vihmc.sensitivity import _operator_batches
    g = deeponet_sens_case("sens_deeponet_small").g
    data = [(torch.from_numpy(g["branch_in"][i]).view(1, 1, -1), torch.from_numpy(g["trunk_in"][g["pts"][i]]).view(1, -1, 2))
            for i in range(g["pts"].shape[0])]
    groups, nb = _operator_batches(data)
    assert nb == len(data) and list(groups) == [(1, g["pts"].shape[1])]
    xt = np.concatenate([t.reshape(-1, 2) for _, t in groups[(1, g["pts"].shape[1])]], 0)
    uniq, inv = np.unique(xt, axis=0, return_inverse=True)
    assert np.array_equal(uniq[inv.reshape(-1)], xt)


def test_sample_points_are_distinct_rows():
    from vihmc.sensitivity import sample_points
    pts = sample_points(50, 10201, 100, seed=3)
    assert pts.shape == (50, 100) and pts.dtype == np.int32
    assert all(len(set(r)) == 100 for r in pts) and pts.min() >= 0 and pts.max() < 10201
    assert np.array_equal(pts, sample_points(50, 10201, 100, seed=3))

"""CPU check of the algebra behind the Gram-form contraction (vi-hmc_amd/csrc/vihmc_gram.hip):
with Zb^ = [Z_b | 1] and Zt^ = [Z_t | b0], the residual form's gradients of the Gaussian NLL
(Operator_network/VI_HMC/main_VI_HMC_burgers.py:157-163 over my_make_func.py:79-82's einsum + bias) equal

    dZb^ = gscale (Zb^ (Zt^T Zt^) - y Zt^),   dZt^ = gscale (Zt^ (Zb^T Zb^) - y^T Zb^),   d/db0 = sum_p dZt^[p][100]

in exact arithmetic (checked in fp64 on random data, several shapes including ragged ones)."""
import numpy as np
import pytest


def residual_form(zb, zt, y, b0, gscale):
    g = gscale * (zb @ zt.T + b0 - y)
    return g @ zt, g.T @ zb, g.sum()


def gram_form(zb, zt, y, b0, gscale):
    n, w = zb.shape
    zbh = np.hstack([zb, np.ones((n, 1))])
    zth = np.hstack([zt, np.full((zt.shape[0], 1), b0)])
    gt = zth.T @ zth
    gb = zbh.T @ zbh
    dzb = gscale * (zbh @ gt - y @ zth)
    dzt = gscale * (zth @ gb - y.T @ zbh)
    return dzb[:, :w], dzt[:, :w], dzt[:, w].sum()


@pytest.mark.parametrize("n,p,w", [(8, 121, 100), (45, 63, 21), (37, 200, 16), (1, 5, 3)])
@pytest.mark.parametrize("loss", ["NLL", "regression"])
def test_gram_form_equals_residual_form(n, p, w, loss):
    rng = np.random.default_rng(n * 1000 + p + w)
    zb = rng.standard_normal((n, w))
    zt = rng.standard_normal((p, w)) * 0.3
    y = rng.standard_normal((n, p))
    b0 = float(rng.standard_normal())
    tau = 0.7
    gscale = -1.0 / tau if loss == "NLL" else -tau
    rb, rt, rs = residual_form(zb, zt, y, b0, gscale)
    gb, gt, gs = gram_form(zb, zt, y, b0, gscale)
    for a, b in ((gb, rb), (gt, rt)):
        assert np.abs(a - b).max() <= 1e-11 * max(1.0, np.abs(b).max())
    assert abs(gs - rs) <= 1e-11 * max(1.0, abs(rs))

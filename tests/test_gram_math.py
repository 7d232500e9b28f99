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


def centred_gram_form(zb, zt, y, b0, gscale, zb0, zt0, b00):
    """The centred form (round 6, DESIGN §3.8, vihmc_gram.hip GramArgs::center): y = S0 + y~ with S0 = B0 T0^T (the
    augmented outputs at the centre weights), dB = Zb^ - B0, dT = Zt^ - T0:
        dZb^ = gscale (dB Gt + B0 Ht - y~ Zt^),  Ht = dT^T Zt^
        dZt^ = gscale (dT Gb + T0 Hb - y~^T Zb^), Hb = dB^T Zb^
        d/db0 = gscale (sum_v (sum_n dB)[v] (sum_p Zt^)[v] + (sum_n B0)[v] (sum_p dT)[v] - sum y~)"""
    n, w = zb.shape
    p = zt.shape[0]
    aug = lambda z, c: np.hstack([z, np.full((z.shape[0], 1), c)])   # noqa: E731
    zbh, zth, b0h, t0h = aug(zb, 1.0), aug(zt, b0), aug(zb0, 1.0), aug(zt0, b00)
    yc = y - b0h @ t0h.T
    db, dt = zbh - b0h, zth - t0h
    gt, ht, gb, hb = zth.T @ zth, dt.T @ zth, zbh.T @ zbh, db.T @ zbh
    dzb = gscale * (db @ gt + b0h @ ht - yc @ zth)
    dzt = gscale * (dt @ gb + t0h @ hb - yc.T @ zbh)
    dsum = gscale * (db.sum(0) @ zth.sum(0) + b0h.sum(0) @ dt.sum(0) - yc.sum())
    return dzb[:, :w], dzt[:, :w], dsum


@pytest.mark.parametrize("n,p,w", [(8, 121, 100), (45, 63, 21), (37, 200, 16), (1, 5, 3)])
def test_centred_gram_form_equals_residual_form(n, p, w):
    rng = np.random.default_rng(n * 7 + p + w)
    zb0 = rng.standard_normal((n, w))
    zt0 = rng.standard_normal((p, w)) * 0.3
    b00 = float(rng.standard_normal())
    zb = zb0 + 0.01 * rng.standard_normal((n, w))          # a chain near the centre
    zt = zt0 + 0.01 * rng.standard_normal((p, w))
    b0 = b00 + 0.01
    y = zb0 @ zt0.T + b00 + 0.05 * rng.standard_normal((n, p))
    gscale = -1.0 / 0.7
    rb, rt, rs = residual_form(zb, zt, y, b0, gscale)
    cb, ct, cs = centred_gram_form(zb, zt, y, b0, gscale, zb0, zt0, b00)
    for a, b in ((cb, rb), (ct, rt)):
        assert np.abs(a - b).max() <= 1e-11 * max(1.0, np.abs(b).max())
    assert abs(cs - rs) <= 1e-10 * max(1.0, abs(rs))

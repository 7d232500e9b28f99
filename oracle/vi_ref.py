"""ORACLE (test infrastructure only) -- one BBB training step of the Bayesian DeepONet restated on the CPU.

Restates the ELBO of Operator_network/VI/main_VI_deeponet.py:58-79 (train_model's inner loop) with
bayesian_model.py:76-114 / layers/BBB/BBBLinear.py:54-78 / metrics.py:13-31,58-60 in float64 torch with
autograd: for each weight draw j, W_j = mu + eps_j * softplus(rho), pred = DeepONet(W_j) (F.linear + act,
einsum, + b), loss_j = gaussian_nll(mean) * train_size + beta * KL(prior || posterior); the step's loss is
the mean over draws. Pinned by tests/golden/vi_deeponet_*.npz (the reference's own train_model).
``log_var`` (learn_noise, noise_type 0: main_VI_deeponet.py:154-156, metrics.py:21-25): the NLL variance is
exp(log_var), a trainable scalar; elbo_step then also returns d loss / d log_var.
Per-item trunk subsets (p < P, utils.py:39-41): NaN entries of y_grid are the grid points an item did not draw;
the NLL and MSE means run over the remaining (item, point) pairs, as the reference's mean over its [B, p] batch.
No reference fixture covers p < P (the golden batches carry the whole grid): that case is parity unpinned.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .deeponet_ref import trunk_feats_np


def _mlp(W, layers, x, act):
    h = x
    for i, l in enumerate(layers):
        w = W[l.w_off:l.w_off + l.n_out * l.n_in].reshape(l.n_out, l.n_in)
        h = F.linear(h, w, W[l.b_off:l.b_off + l.n_out])
        if i < len(layers) - 1:
            h = torch.tanh(h) if act == "tanh" else torch.relu(h)
    return h


def _var(y, noise_var, lv):
    return torch.full_like(y, noise_var) if lv is None else torch.exp(lv) * torch.ones_like(y)


def elbo_step(layout, mu, rho, eps_list, branch_in, trunk_grid, y_grid, beta, train_size, noise_var=1.0,
              prior_mu=0.0, prior_sigma=0.1, act="tanh", log_var=None):
    """(loss, d loss / d mu, d loss / d rho[, d loss / d log_var]) in float64; y_grid [B, P] in trunk_grid order."""
    br, tr, D = layout
    mu_t = torch.tensor(np.asarray(mu, np.float64), requires_grad=True)
    rho_t = torch.tensor(np.asarray(rho, np.float64), requires_grad=True)
    xb = torch.tensor(np.asarray(branch_in, np.float64))
    ft = torch.tensor(trunk_feats_np(trunk_grid))
    y = torch.tensor(np.asarray(y_grid, np.float64))
    m = ~torch.isnan(y)     # p < P (utils.py:39-41): an item's undrawn grid points are NaN and leave the mean
    lv = None if log_var is None else torch.tensor(float(log_var), dtype=torch.float64, requires_grad=True)
    sig = torch.log1p(torch.exp(rho_t))
    sp = torch.tensor(float(prior_sigma), dtype=torch.float64)
    kl = 0.5 * (2 * torch.log(sig / sp) - 1 + (sp / sig) ** 2 + ((mu_t - prior_mu) / sig) ** 2).sum()
    total = 0.0
    for eps in eps_list:
        W = mu_t + torch.tensor(np.asarray(eps, np.float64)) * sig
        pred = _mlp(W, br, xb, act) @ _mlp(W, tr, ft, act).T + W[0]
        nll = F.gaussian_nll_loss(pred[m], y[m], _var(y, noise_var, lv)[m], reduction="mean")
        total = total + nll * train_size + beta * kl
    loss = total / len(eps_list)
    if lv is None:
        gm, gr = torch.autograd.grad(loss, (mu_t, rho_t))
        return float(loss.detach()), gm.numpy(), gr.numpy()
    gm, gr, gl = torch.autograd.grad(loss, (mu_t, rho_t, lv))
    return float(loss.detach()), gm.numpy(), gr.numpy(), float(gl)


def eval_loss(layout, mu, rho, branch_in, trunk_grid, y_grid, beta, size, noise_var=1.0, prior_mu=0.0,
              prior_sigma=0.1, act="tanh", log_var=None):
    """validate_model's loss (eval mode: W = mu) and metrics.mse, float64."""
    br, tr, D = layout
    W = torch.tensor(np.asarray(mu, np.float64))
    sig = torch.log1p(torch.exp(torch.tensor(np.asarray(rho, np.float64))))
    sp = torch.tensor(float(prior_sigma), dtype=torch.float64)
    kl = 0.5 * (2 * torch.log(sig / sp) - 1 + (sp / sig) ** 2 + ((W - prior_mu) / sig) ** 2).sum()
    xb = torch.tensor(np.asarray(branch_in, np.float64))
    ft = torch.tensor(trunk_feats_np(trunk_grid))
    y = torch.tensor(np.asarray(y_grid, np.float64))
    pred = _mlp(W, br, xb, act) @ _mlp(W, tr, ft, act).T + W[0]
    lv = None if log_var is None else torch.tensor(float(log_var), dtype=torch.float64)
    m = ~torch.isnan(y)
    nll = F.gaussian_nll_loss(pred[m], y[m], _var(y, noise_var, lv)[m], reduction="mean")
    return float(nll * size + beta * kl), float(torch.mean((pred - y)[m] ** 2))

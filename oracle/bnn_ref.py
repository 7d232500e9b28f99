"""ORACLE (test infrastructure only) -- BNN (MLP regression) VI-HMC log-posterior restated on the CPU.

Restates ``define_model_log_prob``/``log_prob_func`` of Neural_network/VI_HMC/main_VI_HMC.py:28-153
with ``Functional_Net.functional_model`` (Neural_network/VI_HMC/my_make_func.py:52-73). The same
function with loss='regression', prior std 1 and every parameter sampled is hamiltorch's own
``define_model_log_prob`` used by Neural_network/HMC/main_regression_hmc.py:124-127.

* ``TorchBNNRef`` -- same torch ops (fp32, autograd), including the per-tensor prior slicing quirk.
* ``np_bnn_logp_grad`` -- hand-written forward/backward in numpy (fp64), the kernel spec.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .deeponet_ref import Lin


def mlp_layout(width=(10, 10), bias=True, in_dim=1, out_dim=1) -> Tuple[List[Lin], int]:
    """get_model's nn.Sequential (main_VI_HMC.py:323-333): Linear(1,w0), Linear(w_i,w_i+1)..., Linear(w,1,bias)."""
    dims = [in_dim] + list(width) + [out_dim]
    out, off = [], 0
    for i in range(len(dims) - 1):
        last = i == len(dims) - 2
        has_b = (not last) or bias
        out.append(Lin(off, off + dims[i + 1] * dims[i] if has_b else -1, dims[i + 1], dims[i], not last))
        off += dims[i + 1] * dims[i] + (dims[i + 1] if has_b else 0)
    return out, off


def tensor_sizes(layers) -> List[int]:
    s = []
    for l in layers:
        s.append(l.n_out * l.n_in)
        if l.b_off >= 0:
            s.append(l.n_out)
    return s


class TorchBNNRef:
    def __init__(self, layout, x, y, mu, grad_ind, prior_list=None, loss="NLL", tau_out=0.0025, prior_scale=1.0,
                 act="tanh", load_prior=None):
        """prior_list: per-tensor variances (``Normal(0, tau**0.5)`` per tensor, main_VI_HMC.py:90-91);
        load_prior=(mu0[K], sd0[K]) selects the VI-posterior prior (:87-88)."""
        self.layers, self.D = layout
        self.x = torch.as_tensor(np.asarray(x, np.float32)).reshape(-1, self.layers[0].n_in)
        self.y = torch.as_tensor(np.asarray(y, np.float32)).reshape(-1, self.layers[-1].n_out)
        self.mu = torch.as_tensor(np.asarray(mu, np.float32))
        self.idx = torch.as_tensor(np.asarray(grad_ind, np.int64))
        self.loss, self.tau_out, self.prior_scale = loss, tau_out, prior_scale
        self.act = {"tanh": F.tanh, "relu": F.relu, "sine": torch.sin}[act]
        self.sizes = tensor_sizes(self.layers)
        if load_prior is not None:
            self.dists = None
            self.dist0 = torch.distributions.Normal(torch.as_tensor(np.asarray(load_prior[0], np.float32)),
                                                    torch.as_tensor(np.asarray(load_prior[1], np.float32)))
        else:
            pl = prior_list if prior_list is not None else [1.0] * len(self.sizes)
            self.dists = [torch.distributions.Normal(torch.zeros(()), torch.tensor(float(t)) ** 0.5) for t in pl]
        self.nll = torch.nn.GaussianNLLLoss(reduction="sum")

    def functional_model(self, params):                        # my_make_func.py:52-73
        flat = self.mu.clone()
        flat[self.idx] = params
        x = self.x
        for l in self.layers:
            W = flat[l.w_off:l.w_off + l.n_out * l.n_in].view(l.n_out, l.n_in)
            x = F.linear(x, W, flat[l.b_off:l.b_off + l.n_out] if l.b_off >= 0 else None)
            if l.act:
                x = self.act(x)
        return x

    def log_prob(self, params, predict=False):                 # main_VI_HMC.py:96-151
        l_prior = torch.zeros_like(params[0], requires_grad=True)
        if self.dists is None:
            l_prior = self.dist0.log_prob(params).sum() + l_prior
        else:
            i_prev = 0
            for n, dist in zip(self.sizes, self.dists):
                w = params[i_prev:n + i_prev]
                l_prior = dist.log_prob(w).sum() + l_prior
                i_prev += n
        output = self.functional_model(params)
        if self.loss == "regression":
            ll = -0.5 * self.tau_out * ((output - self.y) ** 2).sum(0)
        elif self.loss == "NLL":
            ll = -self.nll(output, self.y, self.tau_out * torch.ones_like(output))
        else:
            raise NotImplementedError(self.loss)
        lp = ll + l_prior / self.prior_scale
        return (lp, output) if predict else lp

    def logp_grad(self, theta):
        p = torch.as_tensor(np.asarray(theta, np.float32)).clone().requires_grad_()
        lp = self.log_prob(p)
        g, = torch.autograd.grad(lp.sum(), p)
        return float(lp.detach().sum()), g.numpy()


def np_bnn_logp_grad(layout, x, y, mu, grad_ind, theta, prior_mu, prior_sd, loss="NLL", tau_out=0.0025,
                     prior_scale=1.0, act="tanh", dtype=np.float64):
    layers, D = layout
    idx = np.asarray(grad_ind, np.int64)
    th = np.asarray(theta, dtype)
    flat = np.asarray(mu, dtype).copy()
    flat[idx] = th
    h = [np.asarray(x, dtype).reshape(-1, layers[0].n_in)]
    zs = []
    f = {"tanh": np.tanh, "relu": lambda z: np.maximum(z, 0), "sine": np.sin}[act]
    for l in layers:
        W = flat[l.w_off:l.w_off + l.n_out * l.n_in].reshape(l.n_out, l.n_in)
        z = h[-1] @ W.T + (flat[l.b_off:l.b_off + l.n_out] if l.b_off >= 0 else 0)
        zs.append(z)
        h.append(f(z) if l.act else z)
    r = h[-1] - np.asarray(y, dtype).reshape(h[-1].shape)
    if loss == "NLL":
        v = max(float(tau_out), 1e-6)
        ll = -0.5 * (r.size * math.log(v) + np.sum(r * r) / v)
        g = -r / v
    else:
        ll = -0.5 * tau_out * np.sum(r * r)
        g = -tau_out * r
    gflat = np.zeros(D, dtype)
    for j in range(len(layers) - 1, -1, -1):
        l = layers[j]
        if l.act:
            dz = {"tanh": 1 - h[j + 1] ** 2, "relu": (zs[j] > 0).astype(dtype), "sine": np.cos(zs[j])}[act]
            d = g * dz
        else:
            d = g
        gflat[l.w_off:l.w_off + l.n_out * l.n_in] = (d.T @ h[j]).reshape(-1)
        if l.b_off >= 0:
            gflat[l.b_off:l.b_off + l.n_out] = d.sum(0)
        W = flat[l.w_off:l.w_off + l.n_out * l.n_in].reshape(l.n_out, l.n_in)
        g = d @ W
    K = th.shape[0]
    pm = np.broadcast_to(np.asarray(prior_mu, dtype), (K,))
    ps = np.broadcast_to(np.asarray(prior_sd, dtype), (K,))
    lprior = np.sum(-((th - pm) ** 2) / (2 * ps * ps) - np.log(ps) - 0.5 * math.log(2 * math.pi))
    grad = gflat[idx] - (th - pm) / (ps * ps) / prior_scale
    return ll + lprior / prior_scale, grad, h[-1]


def per_tensor_prior_sd(sizes: Sequence[int], K: int, variances: Sequence[float]) -> np.ndarray:
    """std per sampled parameter under the reference's slicing (main_VI_HMC.py:107-112)."""
    sd = np.empty(K)
    i = 0
    for n, t in zip(sizes, variances):
        sd[i:i + n] = math.sqrt(t)
        i += n
        if i >= K:
            break
    return sd

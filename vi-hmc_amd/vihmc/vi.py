"""BBB variational training of the Bayesian DeepONet on the GPU.

Mirrors, with the same names, arguments and return values:
* ``BBB_Linear`` (Operator_network/VI/layers/BBB/BBBLinear.py:14-78) and ``Bayesian_DeepONet``
  (Operator_network/VI/bayesian_model.py:17-114): same parameters, parameter order and initialisation
  draws (made on the CPU generator, as the reference makes them on a CPU-only host);
* ``calculate_kl``, ``get_beta``, ``ELBO`` (Operator_network/VI/metrics.py:13-77), including the
  reference's KL argument order (KL(prior || posterior));
* ``train_model`` / ``validate_model`` / ``mse`` / ``run`` (Operator_network/VI/main_VI_deeponet.py:23-203,
  metrics.py:37-55).

The Gaussian NLL of every batch -- forward and backward through both MLPs and the branch x trunk
contraction over all B x P outputs, for all ``num_ens`` weight draws at once -- is ONE ``vihmc_logp_grad``
call on a full-parameter DeepONet plan (C = num_ens chains, prior weight 0): the HIP kernels of the VI-HMC
path. The reparameterisation W = mu + eps * softplus(rho), the KL term and Adam are D-length elementwise
torch ops on the device; the network enters the autograd graph through ``_EngineNLL``, whose backward is
the engine's gradient. There is no torch forward of the network (no CPU fallback).

Weight-noise draws follow the reference's call order on the CPU generator (per forward: every branch
layer's W_eps then bias_eps, the trunk layers, then the output bias; layers/BBB/BBBLinear.py:55-63,
bayesian_model.py:100), so identical seeds give identical draws. The reference config draws the whole
trunk grid per function (config.py:30, p = 10201): the NLL is a sum over points, so each item's point permutation
(utils.py:39-41) is undone by mapping its points onto the plan's grid order. With p < P every item draws its own
subset: the plan still runs the whole grid, the undrawn (item, point) pairs carry NaN targets that side A counts as
residual 0 (plan options y_masked / lik_count), and the NLL / MSE means run over the B p drawn pairs.
``learn_noise`` with ``noise_type`` 0 (main_VI_deeponet.py:154-156, metrics.py:21-25; off in the reference
config, config.py:45-51): the NLL variance is exp(noise_param), one trainable scalar. The plans are then built
with variance 1, so one evaluation gives 0.5 sum r^2 per draw and its gradient; the log-variance enters in torch
(``elbo_loss``). Not supported: ``noise_type`` 1 (heteroscedastic head, bayesian_model.py:90-92) -- its
einsum("bi,bi->b") takes 2-D branch and trunk outputs, so the reference itself cannot run it on the Burgers
batches (3-D trunk output [B, p, W]); the Cone dataset it serves is out of scope.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import Parameter

from .engine import DeepONetEngine, trunk_features
from .layout import DeepONetSpec
from . import operator as _op

DEFAULT_PRIORS = {"prior_mu": 0, "prior_sigma": 0.1, "posterior_mu_initial": (0, 0.1),
                  "posterior_rho_initial": (-3, 0.1)}


# ------------------------------------------------------------------------------------------------
# metrics.py
# ------------------------------------------------------------------------------------------------
def calculate_kl(mu_q, sig_q, mu_p, sig_p):
    """metrics.py:58-60 (called as KL_DIV(prior_mu, prior_sigma, W_mu, W_sigma) by the layers)."""
    kl = 0.5 * (2 * torch.log(sig_p / sig_q) - 1 + (sig_q / sig_p).pow(2) + ((mu_p - mu_q) / sig_p).pow(2)).sum()
    return kl


def get_beta(batch_idx, m, beta_type, epoch, num_epochs):
    """metrics.py:63-77."""
    if type(beta_type) is float:
        return beta_type
    if beta_type == "Blundell":
        beta = 2 ** (m - (batch_idx + 1)) / (2 ** m - 1)
    elif beta_type == "Soenderby":
        if epoch is None or num_epochs is None:
            raise ValueError("Soenderby method requires both epoch and num_epochs to be passed.")
        beta = min(epoch / (num_epochs // 4), 1)
    elif beta_type == "Standard":
        beta = 1 / m
    else:
        beta = 0
    return beta


class ELBO(nn.Module):
    """metrics.py:13-31: gaussian_nll_loss(mean) * train_size + beta * kl on given predictions (learn_noise:
    noise_param is the log-variance). The training loop evaluates the same quantity through the engine
    (``elbo_loss``)."""

    def __init__(self, learn_noise=False, noise_type=0):
        super().__init__()
        self.learn_noise = learn_noise
        self.noise_type = noise_type

    def forward(self, prediction, target, kl, beta, train_size, noise_param=None):
        assert not target.requires_grad
        if self.learn_noise:
            assert noise_param is not None
            var = torch.exp(noise_param) * torch.ones_like(target) if self.noise_type == 0 else torch.exp(noise_param)
            return F.gaussian_nll_loss(prediction, target, var, reduction="mean") * train_size + beta * kl
        return F.gaussian_nll_loss(prediction.reshape(target.shape), target, noise_param * torch.ones_like(target),
                                   reduction="mean") * train_size + beta * kl


# ------------------------------------------------------------------------------------------------
# layers / model
# ------------------------------------------------------------------------------------------------
def _softplus(rho):
    return torch.log1p(torch.exp(rho))


class BBB_Linear(nn.Module):
    """layers/BBB/BBBLinear.py:14-78: parameters and initialisation (evaluation goes through the engine)."""

    def __init__(self, in_features, out_features, bias=True, priors=None):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.use_bias = bias
        priors = DEFAULT_PRIORS if priors is None else priors
        self.prior_mu = priors["prior_mu"]
        self.prior_sigma = priors["prior_sigma"]
        self.posterior_mu_initial = priors["posterior_mu_initial"]
        self.posterior_rho_initial = priors["posterior_rho_initial"]
        self.W_mu = Parameter(torch.empty((out_features, in_features)))
        self.W_rho = Parameter(torch.empty((out_features, in_features)))
        if not self.use_bias:
            raise NotImplementedError("Bayesian_DeepONet layers have biases (bayesian_model.py:56-72)")
        self.bias_mu = Parameter(torch.empty(out_features))
        self.bias_rho = Parameter(torch.empty(out_features))
        self.reset_parameters()

    def reset_parameters(self):
        self.W_mu.data.normal_(*self.posterior_mu_initial)
        self.W_rho.data.normal_(*self.posterior_rho_initial)
        self.bias_mu.data.normal_(*self.posterior_mu_initial)
        self.bias_rho.data.normal_(*self.posterior_rho_initial)

    def draw_eps(self):
        """The reference forward's draws in its order (BBBLinear.py:56,61): CPU default generator."""
        w = torch.empty(self.W_mu.size()).normal_(0, 1)
        b = torch.empty(self.bias_mu.size()).normal_(0, 1)
        return w, b

    def kl_loss(self):
        kl = calculate_kl(self.prior_mu, self.prior_sigma, self.W_mu, _softplus(self.W_rho))
        kl = kl + calculate_kl(self.prior_mu, self.prior_sigma, self.bias_mu, _softplus(self.bias_rho))
        return kl


class Bayesian_DeepONet(nn.Module):
    """bayesian_model.py:17-114 (noise_type 0). The flat order of mu / rho is the deterministic DeepONet's
    (b, then the branch and trunk layers' weight, bias): means_flattened / stds_flattened of
    Operator_network/VI/sensitivity.py:244-256."""

    def __init__(self, priors, neurons_branch=40, neurons_trunk=40, in_branch=1, in_trunk=1, depth_branch=1,
                 depth_trunk=4, output_neurons=20, activation="relu", noise_type=0, noise_neurons=0, impose_bc=True):
        super().__init__()
        if noise_type:
            raise NotImplementedError("noise_type 1 (heteroscedastic head, bayesian_model.py:90-92) is not supported: "
                                      "the reference's einsum('bi,bi->b') cannot take the Burgers trunk output")
        if activation not in ("relu", "tanh"):
            raise ValueError("activation should be relu or tanh")
        self.neurons_branch, self.neurons_trunk = neurons_branch, neurons_trunk
        self.in_branch, self.in_trunk = in_branch, in_trunk
        self.depth_branch, self.depth_trunk = depth_branch, depth_trunk
        self.output_neurons = output_neurons
        self.noise_type, self.noise_neurons = noise_type, noise_neurons
        self.activation = activation
        self.impose_bc = impose_bc
        self.priors = priors
        self.b_mu = Parameter(torch.empty(1))
        self.b_rho = Parameter(torch.empty(1))
        self.b1 = self._mlp(in_branch, neurons_branch, depth_branch)
        self.b2 = self._mlp(in_trunk, neurons_trunk, depth_trunk)
        self.b_mu.data.normal_(*priors["posterior_mu_initial"])
        self.b_rho.data.normal_(*priors["posterior_rho_initial"])

    def _mlp(self, n_in, width, depth):
        act = nn.ReLU() if self.activation == "relu" else nn.Tanh()
        mods = [BBB_Linear(n_in, width, bias=True, priors=self.priors), act]
        for _ in range(depth - 2):
            mods += [BBB_Linear(width, width, bias=True, priors=self.priors), act]
        mods.append(BBB_Linear(width, self.output_neurons, bias=True, priors=self.priors))
        return nn.Sequential(*mods)

    @property
    def spec(self) -> DeepONetSpec:
        if self.neurons_branch != self.neurons_trunk:
            raise NotImplementedError("branch and trunk widths must match (DeepONetSpec)")
        return DeepONetSpec(self.neurons_branch, self.neurons_trunk, self.in_branch, self.in_trunk, self.depth_branch,
                            self.depth_trunk, self.activation, self.output_neurons, self.impose_bc)

    def bbb_layers(self):
        return [m for m in self.b1 if isinstance(m, BBB_Linear)] + [m for m in self.b2 if isinstance(m, BBB_Linear)]

    def mu_flat(self):
        parts = [self.b_mu.reshape(1)]
        for l in self.bbb_layers():
            parts += [l.W_mu.reshape(-1), l.bias_mu.reshape(-1)]
        return torch.cat(parts)

    def rho_flat(self):
        parts = [self.b_rho.reshape(1)]
        for l in self.bbb_layers():
            parts += [l.W_rho.reshape(-1), l.bias_rho.reshape(-1)]
        return torch.cat(parts)

    def sigma_flat(self):
        return _softplus(self.rho_flat())

    def draw_eps(self):
        """One training forward's weight noise in flat order, drawn in the reference's order (layers, then b)."""
        per_layer = [l.draw_eps() for l in self.bbb_layers()]
        b = torch.empty(self.b_mu.size()).normal_(0, 1)
        parts = [b.reshape(1)]
        for w, bb in per_layer:
            parts += [w.reshape(-1), bb.reshape(-1)]
        return torch.cat(parts)

    def kl(self):
        """forward's kl (bayesian_model.py:106-110): the layers' kl_loss in module order, then b's."""
        kl = 0.0
        for l in self.bbb_layers():
            kl = kl + l.kl_loss()
        pr = self.priors
        return kl + calculate_kl(pr["prior_mu"], pr["prior_sigma"], self.b_mu, _softplus(self.b_rho))


# ------------------------------------------------------------------------------------------------
# the engine inside the autograd graph
# ------------------------------------------------------------------------------------------------
class _EngineNLL(torch.autograd.Function):
    """W [C, D] -> scale * NLL_sum(W_c) [C]; backward = the engine's gradient (one evaluation serves both)."""

    @staticmethod
    def forward(ctx, W, engine, scale):
        lp, g = engine.logp_grad(W.detach())          # prior weight 0: logp = the Gaussian log-likelihood
        ctx.save_for_backward(g)
        ctx.scale = scale
        return -lp * scale

    @staticmethod
    def backward(ctx, go):
        g, = ctx.saved_tensors
        return (-ctx.scale) * go[:, None] * g, None, None


def _ordered_keys(rows: torch.Tensor) -> torch.Tensor:
    """(t, x) fp32 rows [..., 2] -> int64 keys whose signed order is the unsigned order of (bits(t), bits(x))."""
    bits = rows.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return ((bits[..., 0] << 32) | bits[..., 1]) ^ (-(2 ** 63))


def _grid_keys(rows) -> np.ndarray:
    r = np.ascontiguousarray(np.asarray(rows, np.float32).reshape(-1, 2))
    u = r.view(np.uint32).astype(np.uint64)
    return (u[:, 0] << np.uint64(32)) | u[:, 1]


class BatchEngines:
    """Full-parameter plans (one per batch size; the batch data is swapped in with vihmc_plan_set_data),
    NLL variance ``tau_out``, ``max_chains`` weight draws per evaluation, prior weight 0."""

    def __init__(self, spec: DeepONetSpec, trunk_grid, tau_out: float, max_chains: int, device):
        self.spec = spec
        self.grid = np.ascontiguousarray(np.asarray(trunk_grid, np.float32).reshape(-1, 2))
        self.feats = trunk_features(self.grid)
        self.key = _grid_keys(self.grid)
        self.order = np.argsort(self.key, kind="stable")
        self._sorted = {}                   # device -> (sorted ordered keys, order)
        self.tau_out, self.max_chains = float(tau_out), int(max_chains)
        self.device = device
        self._eng: Dict[int, DeepONetEngine] = {}

    @property
    def P(self):
        return self.grid.shape[0]

    def get(self, B: int) -> DeepONetEngine:
        eng = self._eng.get(B)
        if eng is None:
            D = self.spec.n_params
            eng = DeepONetEngine(self.spec, np.zeros((B, self.spec.in_branch), np.float32), self.feats,
                                 np.zeros((B, self.P), np.float32), np.zeros(D, np.float32), np.arange(D), 0.0, 1.0,
                                 "NLL", self.tau_out, float("inf"), max_chains=self.max_chains, device=self.device)
            self._eng[B] = eng
        return eng

    def _work_device(self) -> torch.device:
        dev = torch.device(self.device) if not isinstance(self.device, torch.device) else self.device
        return dev if dev.type == "cuda" and torch.cuda.is_available() else torch.device("cpu")

    def canonical(self, x_trunk, y):
        """(y [B, p] in each item's point order) -> (y_grid [B, P] in the plan's grid order, pair count B p), on the
        plan's device when it has one. Each item's (t, x) rows are located in the grid by their float bit patterns
        (a 64-bit key per row, binary search in the sorted grid keys) and must be distinct grid points; with p < P
        (utils.py:39-41 draws p of the P points per item, without replacement) the grid points an item did not draw
        hold NaN, which the engine's masked plans count as excluded pairs."""
        dev = self._work_device()
        sk = self._sorted.get(dev)
        if sk is None:
            sk = (_ordered_keys(torch.from_numpy(self.grid))[torch.from_numpy(self.order)].to(dev),
                  torch.from_numpy(self.order.astype(np.int64)).to(dev))
            self._sorted[dev] = sk
        skeys, order = sk
        xt = torch.as_tensor(x_trunk).detach().to(dev, torch.float32)
        B = torch.as_tensor(y).shape[0]
        xt = xt.reshape(B, -1, 2)
        p = xt.shape[1]
        if p > self.P:
            raise ValueError(f"an item carries {p} trunk points, the grid has {self.P}")
        yy = torch.as_tensor(y).detach().to(dev, torch.float32).reshape(B, p)
        keys = _ordered_keys(xt).reshape(B, p)
        pos = torch.searchsorted(skeys, keys).clamp_(max=self.P - 1)
        idx = order[pos]
        seen = torch.bincount((idx + self.P * torch.arange(B, device=dev)[:, None]).reshape(-1), minlength=B * self.P)
        if not bool(torch.equal(skeys[pos], keys)) or bool((seen > 1).any()):
            raise ValueError("every trunk point of an item must be a distinct point of the plan's grid")
        yg = torch.full((B, self.P), float("nan"), device=dev) if p < self.P else torch.empty_like(yy)
        return yg.scatter_(1, idx, yy), B * p

    def load(self, batch) -> DeepONetEngine:
        """The batch's branch rows and targets into the plan of its size; p < P marks the plan's targets masked
        (plan options y_masked / lik_count) and ``self.count`` is the batch's (item, point) pair count."""
        xb = torch.as_tensor(batch[0]).detach().to(torch.float32).reshape(-1, self.spec.in_branch)
        eng = self.get(xb.shape[0])
        y, count = self.canonical(batch[1], batch[2])
        eng.set_data(xb, y)
        masked = count < xb.shape[0] * self.P
        # options only on a change: vihmc_plan_option drops the plan's captured graphs (VIHMC_GRAPH=1). The getter of
        # lik_count returns the EFFECTIVE count (N P when the stored value is 0), so it is compared against that.
        for k, v, eff in (("y_masked", 1 if masked else 0, 1 if masked else 0),
                          ("lik_count", count if masked else 0, count)):
            if eng.get_option(k) != eff:
                eng.option(k, v)
        self.count = count
        return eng

    def close(self):
        for e in self._eng.values():
            e.close()
        self._eng.clear()


# ------------------------------------------------------------------------------------------------
# training / validation (main_VI_deeponet.py)
# ------------------------------------------------------------------------------------------------
def _nll_var(log_var):
    """exp(log_var) with F.gaussian_nll_loss's variance clamp (eps 1e-6, applied to the value only)."""
    v = torch.exp(log_var).clone()
    with torch.no_grad():
        v.clamp_(min=1e-6)
    return v


def elbo_loss(model: Bayesian_DeepONet, engines: BatchEngines, batch, beta, train_size, num_ens=1, sample=True,
              log_var=None):
    """sum_j [NLL_mean(pred_j, y) * train_size + beta * kl] / num_ens for one batch (main_VI_deeponet.py:67-75),
    a torch scalar with gradients to the model's mu / rho; the network part is one engine evaluation of all
    num_ens weight draws. ``sample=False`` is eval mode (W = mu, one evaluation). ``log_var`` (learn_noise): the
    trainable log-variance; the engines then run at variance 1 and NLL_mean = 0.5 log v + (0.5 sum r^2) / (v N P)
    (metrics.py:23-25), differentiable in log_var as well."""
    eng = engines.load(batch)
    dev = eng.device
    mu = model.mu_flat()
    if sample:
        eps = torch.stack([model.draw_eps() for _ in range(num_ens)]).to(dev)
        W = mu[None] + eps * model.sigma_flat()[None]
    else:
        num_ens = 1
        W = mu[None]
    count = float(engines.count)                          # (item, point) pairs: B P, or B p with p < P
    if log_var is None:
        nll = _EngineNLL.apply(W, eng, float(train_size) / count)
    else:
        if engines.tau_out != 1.0:
            raise ValueError("learn_noise needs engines built with variance 1 (BatchEngines(..., 1.0, ...))")
        half_sq = _EngineNLL.apply(W, eng, 1.0)              # 0.5 sum r^2 per draw
        v = _nll_var(log_var.to(dev)).reshape(())
        nll = float(train_size) * (0.5 * torch.log(v) + half_sq / (v * count))
    return (nll + beta * model.kl()).sum() / num_ens


def _check_loss(loss):
    if getattr(loss, "noise_type", 0):
        raise NotImplementedError("noise_type 1 (heteroscedastic head) is not supported")


def _log_var(loss, noise_param):
    """The trainable log-variance when the loss learns the noise (metrics.py:21-25), else None (fixed variance =
    the engines' tau_out)."""
    if not getattr(loss, "learn_noise", False):
        return None
    if noise_param is None:
        raise ValueError("learn_noise needs noise_param (the log-variance parameter)")
    return noise_param


def train_model(train_loader, model, loss, optimizer, train_size, num_batches, num_ens=1, beta_type=0.1, epoch=None,
                num_epochs=None, noise_param=None, engines: Optional[BatchEngines] = None):
    """main_VI_deeponet.py:23-81. ``engines`` holds the plans (``BatchEngines(model.spec, grid, noise_param,
    num_ens, device)``); the NLL variance is the engines' tau_out (noise_param of the reference), or, with
    ``loss.learn_noise``, exp(noise_param) (engines at variance 1; noise_param is then a trainable tensor)."""
    _check_loss(loss)
    lv = _log_var(loss, noise_param)
    l_total = 0
    for i, batch_data in enumerate(train_loader):
        model.train()
        optimizer.zero_grad()
        beta = get_beta(i, num_batches, beta_type, epoch, num_epochs)
        l = elbo_loss(model, engines, batch_data, beta, train_size, num_ens, sample=True, log_var=lv)
        l_total += l.item()
        l.backward()
        optimizer.step()
    l_total = l_total / (i + 1)
    return l_total


def validate_model(valid_loader, model, loss, valid_size, beta_type, num_batches, noise_param=None,
                   engines: Optional[BatchEngines] = None):
    """main_VI_deeponet.py:84-127 (eval mode: W = mu)."""
    _check_loss(loss)
    lv = _log_var(loss, noise_param)
    l_total = 0
    for i, batch_data in enumerate(valid_loader):
        model.eval()
        beta = get_beta(i, num_batches, beta_type, None, None)
        with torch.no_grad():
            l = elbo_loss(model, engines, batch_data, beta, valid_size, 1, sample=False, log_var=lv)
        l_total += l.item()
    l_total = l_total / (i + 1)
    return l_total


def mse(data_loader, model, noise_type=0, dataset="Burgers", engines: Optional[BatchEngines] = None):
    """metrics.py:37-55: mean squared error of the eval-mode prediction (W = mu), engine forward."""
    l_total = 0
    for i, batch_data in enumerate(data_loader):
        eng = engines.load(batch_data)
        with torch.no_grad():
            _, out = eng.forward(model.mu_flat().detach()[None].to(eng.device))
        y = engines.canonical(batch_data[1], batch_data[2])[0].to(eng.device)
        # p < P: over each item's own points -- the mask is on the targets only, so a NaN prediction (a diverged
        # model) still gives NaN, as nn.MSELoss does in the reference
        m = ~torch.isnan(y)
        l_total += ((out[0] - y)[m] ** 2).mean().item()
    l_total = l_total / (i + 1)
    return l_total


class BurgersDataSet(torch.utils.data.Dataset):
    """utils.py:27-41: item i = (branch [1, in], trunk rows [p, 2], target [p]) with p random points drawn
    without replacement (a seeded numpy Generator; p = P gives a permutation of the grid)."""

    def __init__(self, branch_in, trunk_in, output, p, seed=0):
        self.x = np.asarray(trunk_in, np.float32).reshape(-1, 2)
        self.u_x = np.asarray(output, np.float32)
        self.f_x = np.asarray(branch_in, np.float32).reshape(self.u_x.shape[0], -1)
        self.p = p
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        return int(self.f_x.shape[0])

    def __getitem__(self, i):
        ind = self.rng.choice(self.x.shape[0], self.p, replace=False)
        return np.expand_dims(self.f_x[i, :], axis=0), self.x[ind], self.u_x[i, ind]


def export_posterior(model: Bayesian_DeepONet, save_loc: str, uid: str):
    """means_flattened_{uid} / stds_flattened_{uid}: 1-D fp32 tensors of mu and softplus(rho) in state_dict
    order (Operator_network/VI/sensitivity.py:244-256) -- the prior files of VI-HMC and of the sensitivity step."""
    os.makedirs(save_loc, exist_ok=True)
    torch.save(model.mu_flat().detach().cpu().contiguous(), f"{save_loc}/means_flattened_{uid}")
    torch.save(model.sigma_flat().detach().cpu().contiguous(), f"{save_loc}/stds_flattened_{uid}")


def run(cfg, train_loader, valid_loader, tr_size, vld_size, trunk_grid, device=None, log=print):
    """main_VI_deeponet.py:130-203 without the checkpoint pickles: Adam + ReduceLROnPlateau over cfg.epochs;
    the posterior of the best validation epoch is exported (``export_posterior``) when cfg.save_loc is set.
    learn_noise (noise_type 0): a trainable log-variance drawn after the model (torch.randn(1), lines 154-156),
    optimised with it; each epoch's metrics then carry exp(noise_param) as a fifth entry (lines 173-175).
    Returns (model, train_metrics)."""
    dev = _op._device("cuda" if device is None else device)
    model = Bayesian_DeepONet(cfg.priors, cfg.width_branch, cfg.width_trunk, cfg.in_branch, cfg.in_trunk,
                              cfg.branch_depth, cfg.trunk_depth, cfg.output_neurons + cfg.noise_neuron,
                              cfg.activation, cfg.noise_type, cfg.noise_neuron,
                              impose_bc=cfg.dataset == "Burgers").to(dev)
    loss = ELBO(cfg.learn_noise, cfg.noise_type)
    _check_loss(loss)
    learn = bool(cfg.learn_noise) and cfg.noise_type == 0
    if learn:
        noise_param = Parameter(torch.randn((1)).to(dev))
        optimizer = torch.optim.Adam(list(model.parameters()) + [noise_param], lr=cfg.lr_start)
        tau = 1.0
    else:
        optimizer = torch.optim.Adam(model.parameters(), lr=cfg.lr_start)
        noise_param = tau = float(cfg.noise_param)
    lr_sched = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, patience=cfg.lr_patience, min_lr=1e-5)
    engines = BatchEngines(model.spec, trunk_grid, tau, cfg.num_ens, dev)
    num_tr, num_val = len(train_loader), len(valid_loader)
    train_metrics = []
    best = float("inf")
    try:
        for epoch in range(cfg.epochs):
            tl = train_model(train_loader, model, loss, optimizer, tr_size, num_tr, cfg.num_ens, cfg.beta_type,
                             noise_param=noise_param, engines=engines)
            vl = validate_model(valid_loader, model, loss, vld_size, cfg.beta_type, num_val, noise_param=noise_param,
                                engines=engines)
            lr_sched.step(vl)
            tm = mse(train_loader, model, engines=engines)
            vm = mse(valid_loader, model, engines=engines)
            alea_unc = float(torch.exp(noise_param.detach()).item()) if learn else 0
            train_metrics.append([tl, vl, tm, vm, alea_unc] if learn else [tl, vl, tm, vm])
            log(f"Epoch: {epoch} \tTraining Loss: {tl:.6f} \tValidation Loss: {vl:.6f} \tTraining MSE: {tm:.6f} "
                f"\tValidation MSE: {vm:.6f} \tNoise: {alea_unc:.6f}")
            if vl <= best:
                best = vl
                if getattr(cfg, "save_loc", None):
                    export_posterior(model, cfg.save_loc, getattr(cfg, "uid", "vi"))
    finally:
        engines.close()
    return model, train_metrics

"""Drop-in replacement of the reference's DeepONet VI-HMC / full-HMC log-prob surface.

Mirrors, with the same names, arguments and return values:
* ``DeepONet`` (Operator_network/VI_HMC/model.py:11-75) -- parameter order and PyTorch default init,
  so ``flatten(net)[grad_ind]`` gives the reference's params_init for the same seed;
* ``define_model_log_prob`` (Operator_network/VI_HMC/main_VI_HMC_burgers.py:27-180) -- the closure
  hamiltorch samples; here backed by the HIP engine (vihmc.engine.DeepONetEngine);
* ``define_split_model_log_prob`` (Operator_network/HMC/main_HMC_splitting.py:209-258) -- one
  full-parameter closure per data shard, prior divided by num_splits;
* ``predict_model`` (main_VI_HMC_burgers.py:183-241) -- batched forward over posterior samples;
* ``get_burgers_data`` (Operator_network/VI_HMC/util.py:461-473) -- the .mat when present, else the
  seeded synthetic problem of the same shapes; ``l2_relative_error`` (post_process_burgers.py:105-121).

The closure returned here is a torch function of ``params`` (autograd.Function whose backward is the
engine's gradient), so any hamiltorch-style caller works; vihmc.samplers recognises it
(``_vihmc_engine``) and drives the batched engine directly.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from .data import deeponet_problem, load_vi_artefacts
from .engine import DeepONetEngine, prior_per_tensor, trunk_features
from .layout import DeepONetSpec


class DeepONet(nn.Module):
    """Same constructor, parameter order and init as the reference DeepONet (model.py:11-75)."""

    def __init__(self, width_branch=40, width_trunk=20, in_branch=1, in_trunk=1, depth_branch=1, depth_trunk=4,
                 activation="relu", output_neurons=None, impose_bc=True):
        super().__init__()
        self.width_branch, self.width_trunk = width_branch, width_trunk
        self.in_branch, self.in_trunk = in_branch, in_trunk
        self.depth_branch, self.depth_trunk = depth_branch, depth_trunk
        self.output_neurons = width_branch if output_neurons is None else output_neurons
        self.activation = activation
        self.b = nn.Parameter(torch.tensor(0.0))
        if activation not in ("relu", "tanh"):
            raise ValueError("Activation can be tanh or relu")
        act = nn.Tanh() if activation == "tanh" else nn.ReLU()
        self.b1 = self._mlp(in_branch, width_branch, depth_branch, act)
        self.b2 = self._mlp(in_trunk, width_trunk, depth_trunk, act)
        self.impose_bc = impose_bc

    def _mlp(self, n_in, width, depth, act):
        mods = [nn.Linear(n_in, width), act]
        for _ in range(depth - 2):
            mods += [nn.Linear(width, width), act]
        mods.append(nn.Linear(width, self.output_neurons))
        return nn.Sequential(*mods)

    @property
    def spec(self) -> DeepONetSpec:
        return DeepONetSpec(self.width_branch, self.width_trunk, self.in_branch, self.in_trunk, self.depth_branch,
                            self.depth_trunk, self.activation, self.output_neurons, self.impose_bc)

    @staticmethod
    def lambda_layer(x):
        return torch.stack([torch.sin(2 * np.pi * x), torch.sin(4 * np.pi * x), torch.cos(2 * np.pi * x),
                            torch.cos(4 * np.pi * x)], dim=2)

    def forward(self, x1, x2):
        x1_out = self.b1(x1)
        if self.impose_bc:
            x_bc = torch.cat([x2[:, :, 0].unsqueeze(dim=2), self.lambda_layer(x2[:, :, 1])], dim=2)
            x2_out = self.b2(x_bc)
        else:
            x2_out = self.b2(x2)
        return torch.einsum("...i,...i->...", x1_out, x2_out) + self.b


def spec_of(model) -> DeepONetSpec:
    if isinstance(model, DeepONetSpec):
        return model
    if hasattr(model, "spec"):
        return model.spec
    # the reference's own DeepONet instance
    return DeepONetSpec(model.width_branch, model.width_trunk, model.in_branch, model.in_trunk, model.depth_branch,
                        model.depth_trunk, "tanh" if isinstance(model.act, nn.Tanh) else "relu", model.output_neurons,
                        getattr(model, "impose_bc", True))


def flatten(model) -> torch.Tensor:
    """util.flatten (Operator_network/VI_HMC/util.py:137-138)."""
    return torch.cat([p.flatten() for p in model.parameters()])


def unflatten(model, flattened_params):
    """util.unflatten (Operator_network/VI_HMC/util.py:141-152)."""
    if flattened_params.dim() != 1:
        raise ValueError("Expecting a 1d flattened_params")
    out, i = [], 0
    for val in model.parameters():
        n = val.nelement()
        out.append(flattened_params[i:i + n].view_as(val))
        i += n
    return out


class _EngineLogProb(torch.autograd.Function):
    """log p(params) with the engine's gradient as its backward (one evaluation serves both)."""

    @staticmethod
    def forward(ctx, params, engine, shape):
        lp, g = engine.logp_grad(params.detach().reshape(1, -1))
        ctx.save_for_backward(g[0].to(params.device))
        return lp[0].to(params.device).reshape(shape)

    @staticmethod
    def backward(ctx, grad_out):
        g, = ctx.saved_tensors
        return grad_out.sum() * g, None, None


def make_closure(engine, predict=False, out_shape=(), resample=None):
    def log_prob_func(params, *args):
        if len(args) != 0:                    # main_VI_HMC_burgers.py:91-94 (fsample)
            if resample is not None:
                resample()
            print("Sampled from learned parameter distributions")
            return None
        if predict:
            with torch.no_grad():
                lp, out = engine.forward(params.detach().reshape(1, -1))
            return lp[0].to(params.device).reshape(out_shape), out[0].to(params.device)
        if params.requires_grad and torch.is_grad_enabled():
            return _EngineLogProb.apply(params, engine, out_shape)
        return engine.logp(params.detach().reshape(1, -1))[0].to(params.device).reshape(out_shape)

    log_prob_func._vihmc_engine = engine
    return log_prob_func


def _device(device):
    d = torch.device(device) if not isinstance(device, torch.device) else device
    if d.type != "cuda":
        d = torch.device("cuda", torch.cuda.current_device())   # the engine only runs on a HIP device
    return d


def _prior_from_tau_list(cfg, tau_list, K):
    if getattr(cfg, "load_prior", False):            # Normal(tau_list[0], tau_list[1]) (:75-78)
        return np.asarray(torch.as_tensor(tau_list[0]).cpu(), np.float32), np.asarray(
            torch.as_tensor(tau_list[1]).cpu(), np.float32)
    tau = float(torch.as_tensor(tau_list[0]))        # Normal(0, tau**0.5) (:79-81)
    return 0.0, tau ** 0.5


def define_model_log_prob(model, model_loss, tr_data, tau_list, tau_out, predict=False, prior_scale=1.0,
                          device="cpu", cfg=None, mu=None, sigma=None, grad_ind=None, max_chains=1, full=False):
    """main_VI_HMC_burgers.py:27-180. Reads ``means_flattened_{uid}``, ``stds_flattened_{uid}`` and
    ``gradient_indices_{uid}.npy`` from ``cfg.prior_file`` unless mu/sigma/grad_ind are given.
    ``full=True`` (or ``mu=None`` with no artefact file) selects full-parameter HMC (the ``mus=None``
    branch, Operator_network/HMC/main_HMC_splitting.py:79-206): no artefacts are read, and
    ``cfg.load_prior`` then means tau_list = [means[D], stds[D]] (main_HMC_splitting.py:341-345)."""
    spec = spec_of(model)
    if full:
        mu = grad_ind = None
    elif mu is None and cfg is not None and getattr(cfg, "prior_file", None):
        mu, sigma, gi = load_vi_artefacts(cfg.prior_file, cfg.prior_uid)
        grad_ind = gi if grad_ind is None else grad_ind
    full = mu is None
    if full:
        mu = np.zeros(spec.n_params, np.float32)
        grad_ind = np.arange(spec.n_params)
    grad_ind = np.asarray(grad_ind, np.int64)
    x1, x2, y = tr_data
    pm, ps = _prior_from_tau_list(cfg, tau_list, grad_ind.size)
    loss = model_loss
    if loss not in ("NLL", "regression"):
        raise NotImplementedError(f"model_loss {model_loss!r}")
    xb = np.asarray(torch.as_tensor(x1).cpu()).reshape(-1, spec.in_branch)
    feats, yy = trunk_features(torch.as_tensor(x2).cpu()), np.asarray(torch.as_tensor(y).cpu())
    # cfg.sample_data (:127-137): every non-predict evaluation sees cfg.p trunk rows drawn with random.sample
    p_sub = int(cfg.p) if getattr(cfg, "sample_data", False) and not predict else None
    if p_sub is not None and not 0 < p_sub <= feats.shape[0]:
        raise ValueError(f"cfg.p={p_sub} must be in [1, {feats.shape[0]}] (the trunk grid size)")

    def build(w, dev):
        e = DeepONetEngine(spec, xb, feats if p_sub is None else feats[:p_sub],
                           yy if p_sub is None else yy[:, :p_sub], w, grad_ind, pm, ps, loss, tau_out, prior_scale,
                           max_chains=max_chains, device=dev)
        if p_sub is not None:
            e.sample_data(feats, yy, p_sub)
        return e

    eng = build(mu, _device(device))

    def resample():
        if sigma is None:
            return
        w = torch.normal(torch.as_tensor(mu), torch.as_tensor(sigma)).numpy()
        eng.close()
        new = build(w, eng.device)
        eng.__dict__.update(new.__dict__)
        new._plan = None                      # ownership moved into `eng`

    return make_closure(eng, predict, (), resample)


def define_split_model_log_prob(model, model_loss, train_loader, num_splits, tau_list, tau_out, predict=False,
                                device="cpu", verbose=True, cfg=None, max_chains=1):
    """Operator_network/HMC/main_HMC_splitting.py:209-258: full-parameter closures over data shards,
    each with prior_scale=num_splits. ``cfg`` carries load_prior / sample_data as in the reference's
    define_model_log_prob (:115-206); the VI artefact files are never read on this path."""
    out = []
    for i, data in enumerate(train_loader):
        if i > num_splits - 1:
            break
        out.append(define_model_log_prob(model, model_loss, data, tau_list, tau_out, predict=predict,
                                         prior_scale=num_splits, device=device, cfg=cfg, full=True,
                                         max_chains=max_chains))
    if verbose:
        print("Number of splits: ", len(out), " , each of batch size ", train_loader[0][0].shape[0], "\n")
    return out


def define_model_log_prob_nuts(model, model_loss, tr_data, params_flattened_list, params_shape_list, tau_list,
                               tau_out, predict=False, prior_scale=1.0, device="cpu", cfg=None, max_chains=1):
    """Operator_network/HMC/NUTS_DeepOnets.py:78-200: full-parameter DeepONet closure with a per-tensor prior.
    Reference quirk kept: without cfg.load_prior the prior of tensor i is
    Normal(0, tau_list[i] * 0.5) -- tau used as a std and halved (:128-132); with cfg.load_prior it is
    Normal(tau_list[0], tau_list[1]) over all D parameters."""
    spec = spec_of(model)
    D = spec.n_params
    if getattr(cfg, "load_prior", False):
        pm = np.asarray(torch.as_tensor(tau_list[0]).cpu(), np.float32)
        ps = np.asarray(torch.as_tensor(tau_list[1]).cpu(), np.float32)
    else:
        taus = [float(t) for t in torch.as_tensor(torch.stack([torch.as_tensor(t) for t in tau_list])).cpu()]
        if len(taus) != len(params_flattened_list) or sum(params_flattened_list) != D:
            raise ValueError("tau_list / params_flattened_list must have one entry per parameter tensor")
        pm = 0.0
        ps = prior_per_tensor(list(params_flattened_list), D, [0.5 * t for t in taus])
    x1, x2, y = tr_data
    if model_loss not in ("NLL", "regression"):
        raise NotImplementedError(f"model_loss {model_loss!r}")
    eng = DeepONetEngine(spec, np.asarray(torch.as_tensor(x1).cpu()).reshape(-1, spec.in_branch),
                         trunk_features(torch.as_tensor(x2).cpu()), np.asarray(torch.as_tensor(y).cpu()),
                         np.zeros(D, np.float32), np.arange(D), pm, ps, model_loss, tau_out, prior_scale,
                         max_chains=max_chains, device=_device(device))
    return make_closure(eng, predict, ())


def predict_model(model, samples, test_loader=None, model_loss="NLL", tau_out=1., tau_list=None, cfg=None,
                  mu=None, sigma=None, grad_ind=None, batch=16, device=None):
    """main_VI_HMC_burgers.py:183-241: (predictions [S, N, P], list of S log-probs), evaluated in
    batches of ``batch`` samples per engine call."""
    samples = samples if torch.is_tensor(samples) else torch.stack(list(samples))
    if tau_list is None:
        tau_list = [torch.tensor(1.)]
    dev = _device(device if device is not None else samples.device)
    S = samples.shape[0]
    b = max(1, min(batch, S))
    f = define_model_log_prob(model, model_loss, test_loader, tau_list, tau_out, predict=True, device=dev, cfg=cfg,
                              mu=mu, sigma=sigma, grad_ind=grad_ind, max_chains=b)
    eng = f._vihmc_engine
    preds, lps = [], []
    with torch.no_grad():
        for s in range(0, S, b):
            lp, out = eng.forward(samples[s:s + b].to(dev))
            preds.append(out.to(samples.device))
            lps.extend(lp.to(samples.device).unbind(0))
    return torch.cat(preds), lps


def get_burgers_data(cfg, mat_path: str = "../Data/DeepOnet_data.mat", seed: int = 0):
    """(train, valid) tuples (branch [N,1,101], trunk [1,P,2], y [N,P]) as util.get_burgers_data;
    the seeded synthetic problem when the .mat is absent (it is not shipped with the reference)."""
    if os.path.exists(mat_path):
        import scipy.io
        m = scipy.io.loadmat(mat_path)

        def part(lo, hi):
            return (torch.tensor(np.expand_dims(m["branch_in"][lo:hi].astype(np.float32), axis=1)),
                    torch.tensor(np.expand_dims(m["trunk_in"].astype(np.float32), axis=0)),
                    torch.tensor(m["solution"][lo:hi].astype(np.float32)))
        return part(0, cfg.N_train), part(cfg.N_train, cfg.N_train + cfg.N_valid)
    p = deeponet_problem(seed=seed, n=cfg.N_train + cfg.N_valid, k=None)
    n = cfg.N_train

    def part(lo, hi):
        return (torch.from_numpy(p.branch_in[lo:hi]), torch.from_numpy(p.trunk_in), torch.from_numpy(p.y[lo:hi]))
    return part(0, n), part(n, n + cfg.N_valid)


def l2_relative_error(y_true, y_pred):
    """post_process_burgers.py:105-121 (per-function relative L2 error)."""
    if y_true.shape != y_pred.shape:
        raise ValueError("Shape mismatch")
    return np.linalg.norm(y_true - y_pred, axis=1) / np.linalg.norm(y_true, axis=1)

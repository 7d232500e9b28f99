"""Drop-in replacement of the reference's BNN (MLP regression) VI-HMC / HMC log-prob surface.

Mirrors Neural_network/VI_HMC/main_VI_HMC.py (``get_model`` :297-334, ``define_model_log_prob``
:28-153, ``predict_model`` :156-259, ``get_data`` :262-294) and hamiltorch's own
``define_model_log_prob`` / ``sample_model`` / ``predict_model`` used by
Neural_network/HMC/main_regression_hmc.py:102-176 (restated: prior N(0, tau^-1/2) per tensor,
'regression' ll = -0.5*tau_out*sum r^2, all parameters sampled). The log-prob runs on the
wave-per-chain HIP kernel (vihmc.engine.MLPEngine).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from .data import bnn_data, load_vi_artefacts
from .engine import MLPEngine, prior_per_tensor
from .layout import MLPSpec
from .operator import _device, make_closure
from . import samplers


class Sin(nn.Module):
    def forward(self, x):
        return torch.sin(x)


def get_model(cfg, bias_on: bool = True) -> nn.Sequential:
    """main_VI_HMC.py:297-334 (same module order, so the same init for the same seed)."""
    acts = {"relu": nn.ReLU, "tanh": nn.Tanh, "sine": Sin}
    if cfg.act not in acts:
        raise ValueError("Activation should be relu, sine or tanh")
    act_fn = acts[cfg.act]()
    mods = [nn.Linear(1, cfg.width[0]), act_fn]
    i = -1
    for i in range(len(cfg.width) - 1):
        mods += [nn.Linear(cfg.width[i], cfg.width[i + 1]), act_fn]
    mods.append(nn.Linear(cfg.width[i + 1], 1, bias=bias_on))
    return nn.Sequential(*mods)


def spec_of(model) -> MLPSpec:
    if isinstance(model, MLPSpec):
        return model
    lins = [m for m in model if isinstance(m, nn.Linear)]
    act = "tanh"
    for m in model:
        if isinstance(m, nn.ReLU):
            act = "relu"
        elif isinstance(m, nn.Tanh):
            act = "tanh"
        elif type(m).__name__ == "Sin":
            act = "sine"
    return MLPSpec(width=tuple(l.out_features for l in lins[:-1]), act=act, bias=lins[-1].bias is not None,
                   in_dim=lins[0].in_features, out_dim=lins[-1].out_features)


def flatten(model) -> torch.Tensor:
    return torch.cat([p.flatten() for p in model.parameters()])


def _np(t):
    return np.asarray(torch.as_tensor(t).detach().cpu(), np.float32)


def define_model_log_prob(model, model_loss, x, y, params_flattened_list, params_shape_list, prior_list, tau_out,
                          predict=False, prior_scale=1.0, device="cpu", dt_string=None, grad_ind=None, cfg=None,
                          mu=None, sigma=None, max_chains=1):
    """main_VI_HMC.py:28-153. mu/sigma default to cfg's ``means_flattened_{uid}``/``stds_flattened_{uid}``."""
    spec = spec_of(model)
    if mu is None:
        mu, sigma, gi = load_vi_artefacts(cfg.prior_file, cfg.prior_uid)
        grad_ind = gi if grad_ind is None else grad_ind
    grad_ind = np.asarray(grad_ind, np.int64)
    K = grad_ind.size
    if getattr(cfg, "load_prior", False):
        pm, ps = _np(prior_list[0]), _np(prior_list[1])
    else:
        pm = 0.0
        ps = prior_per_tensor(list(params_flattened_list), K, [float(torch.as_tensor(t)) ** 0.5 for t in prior_list])
    eng = MLPEngine(spec, _np(x), _np(y), mu, grad_ind, pm, ps, model_loss, tau_out, prior_scale, max_chains,
                    device=_device(device))
    shape = (1,) if model_loss == "regression" else ()
    return make_closure(eng, predict, shape)


def define_model_log_prob_hamiltorch(model, model_loss, x, y, params_flattened_list, params_shape_list, tau_list,
                                     tau_out, normalizing_const=1., predict=False, prior_scale=1.0, device="cpu",
                                     max_chains=1):
    """hamiltorch.define_model_log_prob for the plain-HMC BNN (config 1): every parameter sampled,
    prior N(0, tau^-1/2) per tensor (precision tau)."""
    spec = spec_of(model)
    D = spec.n_params
    ps = prior_per_tensor(list(params_flattened_list), D, [float(t) ** -0.5 for t in torch.as_tensor(tau_list)])
    eng = MLPEngine(spec, _np(x), _np(y), np.zeros(D, np.float32), np.arange(D), 0.0, ps, model_loss, tau_out,
                    prior_scale, max_chains, device=_device(device))
    shape = (1,) if model_loss == "regression" else ()
    return make_closure(eng, predict, shape)


def sample_model(model, x, y, params_init, model_loss="regression", num_samples=10, num_steps_per_sample=10,
                 step_size=0.1, burn=0, inv_mass=None, normalizing_const=1., sampler=samplers.Sampler.HMC,
                 integrator=samplers.Integrator.IMPLICIT, debug=False, tau_out=1., tau_list=None,
                 desired_accept_rate=0.8, verbose=False, **unused):
    """hamiltorch.sample_model as called at Neural_network/HMC/main_regression_hmc.py:124-127."""
    sizes = [p.nelement() for p in model.parameters()]
    shapes = [p.shape for p in model.parameters()]
    if tau_list is None:
        tau_list = torch.ones(len(sizes))
    f = define_model_log_prob_hamiltorch(model, model_loss, x, y, sizes, shapes, tau_list, tau_out, normalizing_const,
                                         device=params_init.device)
    return samplers.sample(f, params_init, num_samples=num_samples, num_steps_per_sample=num_steps_per_sample,
                           step_size=step_size, burn=burn, inv_mass=inv_mass, sampler=sampler, integrator=integrator,
                           debug=debug, desired_accept_rate=desired_accept_rate, verbose=verbose)


def _predict(eng, samples, batch):
    preds, lps = [], []
    with torch.no_grad():
        for s in range(0, samples.shape[0], batch):
            lp, out = eng.forward(samples[s:s + batch].to(eng.device))
            preds.append(out.to(samples.device))
            lps.extend(lp.to(samples.device).unbind(0))
    return torch.cat(preds), lps


def predict_model(model, samples, x=None, y=None, test_loader=None, model_loss="multi_class_linear_output",
                  tau_out=1., prior_list=None, verbose=False, dt_string=None, grad_ind=None, cfg=None, mu=None,
                  sigma=None, batch=64):
    """main_VI_HMC.py:156-259 (x/y form): (predictions [S, N, 1], list of S log-probs)."""
    samples = samples if torch.is_tensor(samples) else torch.stack(list(samples))
    if x is None or y is None:
        raise RuntimeError("Val data not defined (i.e. arguments x, y, val_loader are all not defined)")
    sizes = [p.nelement() for p in model.parameters()]
    shapes = [p.shape for p in model.parameters()]
    if prior_list is None:
        prior_list = [torch.tensor(1.)] * len(sizes)
    b = max(1, min(batch, samples.shape[0]))
    f = define_model_log_prob(model, model_loss, x, y, sizes, shapes, prior_list, tau_out, predict=True,
                              device=samples.device, grad_ind=grad_ind, cfg=cfg, mu=mu, sigma=sigma, max_chains=b)
    return _predict(f._vihmc_engine, samples, b)


def predict_model_hamiltorch(model, samples, x, y, model_loss="regression", tau_out=1., tau_list=None, batch=64):
    """hamiltorch.predict_model as called at Neural_network/HMC/main_regression_hmc.py:153-155."""
    samples = samples if torch.is_tensor(samples) else torch.stack(list(samples))
    sizes = [p.nelement() for p in model.parameters()]
    if tau_list is None:
        tau_list = torch.ones(len(sizes))
    b = max(1, min(batch, samples.shape[0]))
    f = define_model_log_prob_hamiltorch(model, model_loss, x, y, sizes, None, tau_list, tau_out, predict=True,
                                         device=samples.device, max_chains=b)
    return _predict(f._vihmc_engine, samples, b)


def get_data(cfg=None, path: Optional[str] = None):
    """(x_train, y_train, x_val, y_val) torch tensors (main_VI_HMC.py:262-294)."""
    tau = getattr(cfg, "tau_out", 0.0025) if cfg is not None else 0.0025
    return tuple(torch.from_numpy(a) for a in bnn_data(path, tau_out=tau))

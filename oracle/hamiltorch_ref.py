"""ORACLE (test infrastructure only) -- scalar restatement of hamiltorch's HMC sampler.

hamiltorch (``requirements.txt:1``, ``git+https://github.com/AdamCobb/hamiltorch``, no pinned
commit) is an un-vendored third-party dependency that is absent from this container; its published
algorithm is restated here for ``Sampler.HMC`` / ``Sampler.HMC_NUTS``
(dual-averaging step size during burn) with ``Integrator.IMPLICIT`` (plain leapfrog) and
``Integrator.SPLITTING`` (Neal's split Hamiltonian over data shards), identity or diagonal mass.
Reference call sites: Operator_network/VI_HMC/main_VI_HMC_burgers.py:286-287,
Neural_network/VI_HMC/main_VI_HMC.py:379-380, Operator_network/HMC/main_HMC_splitting.py:361-369.

Sampler parity is UNPINNED: no reference test or fixture holds hamiltorch outputs. This
restatement is the checker for vihmc.samplers on identical RNG streams.

RNG: momentum = Normal(0, 1 [or mass**0.5]).sample() on the params' device generator, then the
accept draw torch.rand(1) on the CPU generator -- both from ``generator`` here when given (one CPU
stream per chain), else the global generators as hamiltorch does.
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Sequence, Union

import torch

HMC, HMC_NUTS = "HMC", "HMC_NUTS"
IMPLICIT, SPLITTING = "IMPLICIT", "SPLITTING"


class LogProbError(Exception):
    pass


def has_nan_or_inf(value) -> bool:
    if torch.is_tensor(value):
        value = torch.sum(value)
        return bool(torch.isnan(value)) or bool(torch.isinf(value))
    value = float(value)
    return value in (float("inf"), float("-inf")) or value != value


def _grad(fn, p):
    p = p.detach().requires_grad_()
    lp = fn(p)
    return torch.autograd.grad(lp.sum() if lp.dim() else lp, p)[0]


def gibbs(params, mass=None, generator=None):
    std = torch.ones_like(params) if mass is None else mass ** 0.5
    return torch.normal(torch.zeros_like(params), std, generator=generator)


def hamiltonian(params, momentum, log_prob_func, inv_mass=None):
    fns = log_prob_func if isinstance(log_prob_func, list) else [log_prob_func]
    log_prob = 0.0
    for f in fns:
        lp = f(params)
        if has_nan_or_inf(lp):
            raise LogProbError()
        log_prob = log_prob + lp
    potential = -log_prob
    kinetic = 0.5 * torch.dot(momentum, momentum) if inv_mass is None else 0.5 * torch.dot(momentum, inv_mass * momentum)
    return potential + kinetic


def leapfrog(params, momentum, log_prob_func, steps, step_size, inv_mass=None, integrator=IMPLICIT):
    if integrator != SPLITTING:
        momentum = momentum + 0.5 * step_size * _grad(log_prob_func, params)
        p_grad = None
        ret_params, ret_momenta = [], []
        for _ in range(steps):
            params = params + step_size * momentum if inv_mass is None else params + step_size * inv_mass * momentum
            p_grad = _grad(log_prob_func, params)
            momentum = momentum + step_size * p_grad
            ret_params.append(params.clone())
            ret_momenta.append(momentum.clone())
        ret_momenta[-1] = ret_momenta[-1] - 0.5 * step_size * p_grad.clone()
        return ret_params, ret_momenta
    fns = log_prob_func
    M = len(fns)
    ret_params, ret_momenta = [], []
    params = params.detach()
    for _ in range(steps):
        for m in range(M):
            momentum = momentum + 0.5 * step_size * _grad(fns[m], params)
            if m < M - 1:
                params = params + (step_size / (2 * (M - 1))) * momentum
        for m in reversed(range(M)):
            momentum = momentum + 0.5 * step_size * _grad(fns[m], params)
            if m > 0:
                params = params + (step_size / (2 * (M - 1))) * momentum
        ret_params.append(params)
        ret_momenta.append(momentum)
    return ret_params, ret_momenta


def adaptation(rho, t, step_size_init, H_t, eps_bar, desired_accept_rate=0.8):
    t = t + 1
    if has_nan_or_inf(torch.tensor([rho])):
        alpha = 0
    else:
        alpha = min(1., float(torch.exp(torch.FloatTensor([rho]))))
    mu = float(torch.log(10 * torch.FloatTensor([step_size_init])))
    gamma, t0, kappa = 0.05, 10, 0.75
    H_t = (1 - (1 / (t + t0))) * H_t + (1 / (t + t0)) * (desired_accept_rate - alpha)
    x_new = mu - (t ** 0.5) / gamma * H_t
    step_size = float(torch.exp(torch.FloatTensor([x_new])))
    x_new_bar = t ** -kappa * x_new + (1 - t ** -kappa) * torch.log(torch.FloatTensor([eps_bar]))
    eps_bar = float(torch.exp(x_new_bar))
    return step_size, eps_bar, H_t


def sample(log_prob_func: Union[Callable, List[Callable]], params_init, num_samples=10, num_steps_per_sample=10,
           step_size=0.1, burn=0, inv_mass=None, sampler=HMC, integrator=IMPLICIT, desired_accept_rate=0.8,
           generator: Optional[torch.Generator] = None, return_stats=False):
    if params_init.dim() != 1:
        raise RuntimeError("params_init must be a 1d tensor.")
    if burn >= num_samples:
        raise RuntimeError("burn must be less than num_samples.")
    NUTS = sampler == HMC_NUTS
    if NUTS:
        if burn == 0:
            raise RuntimeError("burn must be greater than 0 for NUTS.")
        step_size_init, H_t, eps_bar = step_size, 0., 1.
    mass = None if inv_mass is None else 1 / inv_mass
    params = params_init.clone().requires_grad_()
    param_burn_prev = params_init.clone()
    ret_params = [params.clone()]
    num_rejected = 0
    accepts = []
    step_sizes = []
    rhos, logus = [], []
    for n in range(num_samples):
        try:
            momentum = gibbs(params, mass, generator)
            ham = hamiltonian(params, momentum, log_prob_func, inv_mass)
            lp_params, lp_momenta = leapfrog(params, momentum, log_prob_func, num_steps_per_sample, step_size,
                                             inv_mass, integrator)
            params = lp_params[-1].detach().requires_grad_()
            momentum = lp_momenta[-1]
            new_ham = hamiltonian(params, momentum, log_prob_func, inv_mass)
            rho = min(0., float(-new_ham + ham))
            logu = torch.log(torch.rand(1, generator=generator))
            rhos.append(rho)
            logus.append(float(logu))
            if rho >= logu:
                accepts.append(True)
                if n > burn:
                    ret_params.append(lp_params[-1])
                else:
                    param_burn_prev = lp_params[-1].clone()
            else:
                accepts.append(False)
                num_rejected += 1
                if n > burn:
                    params = ret_params[-1]
                    ret_params.append(ret_params[-1])
                else:
                    params = param_burn_prev.clone()
            if NUTS and n <= burn:
                if n < burn:
                    step_size, eps_bar, H_t = adaptation(rho, n, step_size_init, H_t, eps_bar, desired_accept_rate)
                if n == burn:
                    step_size = eps_bar
        except LogProbError:
            rhos.append(float("nan"))
            logus.append(float("nan"))
            accepts.append(False)
            num_rejected += 1
            params = ret_params[-1].detach().requires_grad_()
            if NUTS and n <= burn:
                step_size, eps_bar, H_t = adaptation(float("nan"), n, step_size_init, H_t, eps_bar,
                                                     desired_accept_rate)
            if NUTS and n == burn:
                step_size = eps_bar
        step_sizes.append(step_size)
    out = [t.detach() for t in ret_params]
    if return_stats:
        return out, dict(num_rejected=num_rejected, accepts=accepts, step_sizes=step_sizes, rhos=rhos, logus=logus)
    return out

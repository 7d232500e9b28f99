"""hamiltorch-compatible HMC sampler, batched over chains and resident on the GPU.

The reference hands a scalar ``log_prob_func`` to the un-vendored ``hamiltorch.samplers.sample``
(call sites: Operator_network/VI_HMC/main_VI_HMC_burgers.py:286-287,
Neural_network/VI_HMC/main_VI_HMC.py:379-380, Operator_network/HMC/main_HMC_splitting.py:361-369).
This module keeps that algorithm -- Gibbs momentum, leapfrog (or Neal's split integrator), Metropolis
accept, the dual-averaging step size of ``Sampler.HMC_NUTS`` -- and its exact bookkeeping (what is
stored during / after burn, what a rejection reverts to, ``LogProbError`` = non-finite log-prob =>
reject without storing), restated in SURVEY.md Appendix A and oracle/hamiltorch_ref.py, but runs C
chains at once:

* state (theta, logp, grad) lives in [C, K] device tensors; the accept decision is a device-side
  ``torch.where``, so there is no host synchronisation per sample (except during NUTS burn-in, where
  the step-size adaptation is host arithmetic per chain, as in hamiltorch);
* momenta and accept uniforms come from one CPU ``torch.Generator`` per chain (seeded per chain, so a
  chain's draws do not depend on how chains are sharded over GPUs), drawn in hamiltorch's order
  (normal(K) then rand(1)); ``rng="global"`` reproduces hamiltorch's use of the global generators;
* the gradient at the start of a trajectory is the one computed at its end point by the previous
  trajectory (or at the revert target), which the deterministic HIP engine makes bit-identical to a
  recomputation: L gradient evaluations per sample instead of hamiltorch's L+1 (reuse_endpoint_grad).

Elementwise updates use the same op sequence as hamiltorch (``p = p + fp32(eps)*g`` as a separate
multiply and add, no fused FMA), so trajectories match the oracle to the engine's fp32 tolerance.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from enum import Enum
from typing import Callable, List, Optional, Sequence, Union

import torch


class Sampler(Enum):
    HMC = 1
    RMHMC = 2
    HMC_NUTS = 3


class Integrator(Enum):
    EXPLICIT = 1
    IMPLICIT = 2
    S3 = 3
    SPLITTING = 4
    SPLITTING_RAND = 5
    SPLITTING_KMID = 6


class LogProbError(Exception):
    """Non-finite log-probability (reference util.py:107-119); the sampler treats it as a rejection."""


# ------------------------------------------------------------------------------------------------
# evaluators: theta [C, K] -> (logp [C], grad [C, K])
# ------------------------------------------------------------------------------------------------
class EngineEvaluator:
    """Batched HIP engine (vihmc.engine.*Engine)."""

    def __init__(self, engine):
        self.engine = engine
        self.K = engine.K
        self.device = engine.device
        self.n_grad = 0
        self.n_value = 0

    def logp_grad(self, theta):
        self.n_grad += theta.shape[0]
        return self.engine.logp_grad(theta)

    def logp(self, theta):
        self.n_value += theta.shape[0]
        return self.engine.logp(theta)

    def grad(self, theta):
        """gradient only (the leapfrog's inner steps, whose log-prob hamiltorch discards): vihmc_grad"""
        self.n_grad += theta.shape[0]
        if hasattr(self.engine, "grad"):
            return self.engine.grad(theta)
        return self.engine.logp_grad(theta)[1]

    @property
    def fused_trajectory(self) -> bool:
        """Engines run a whole leapfrog trajectory per call (_Engine.trajectory / vihmc_trajectory: one launch for
        BNN plans, the updates fused into the gradient gather for DeepONet plans); False = step-by-step path."""
        return hasattr(self.engine, "trajectory") and getattr(self.engine, "fused_trajectory", True)

    def trajectory(self, theta, p, g, eps, L, inv_mass=None):
        self.n_grad += theta.shape[0] * L
        return self.engine.trajectory(theta, p, g, eps, L, inv_mass)


class AutogradEvaluator:
    """Any scalar torch closure ``f(params[K]) -> logp`` (the reference's own contract), one chain
    at a time through torch.autograd -- the generic fallback for user-defined log-probs."""

    def __init__(self, fn: Callable, K: int, device):
        self.fn, self.K, self.device = fn, K, torch.device(device)
        self.n_grad = 0
        self.n_value = 0

    def logp_grad(self, theta):
        lps, gs = [], []
        for c in range(theta.shape[0]):
            p = theta[c].detach().clone().requires_grad_()
            lp = self.fn(p)
            lp = lp.sum() if lp.dim() else lp
            g, = torch.autograd.grad(lp, p)
            lps.append(lp.detach().reshape(()))
            gs.append(g)
        self.n_grad += theta.shape[0]
        return torch.stack(lps).to(torch.float32), torch.stack(gs).to(torch.float32)

    def grad(self, theta):
        return self.logp_grad(theta)[1]

    def logp(self, theta):
        with torch.no_grad():
            out = torch.stack([self.fn(theta[c]).sum().reshape(()) for c in range(theta.shape[0])])
        self.n_value += theta.shape[0]
        return out.to(torch.float32)


def evaluator_for(log_prob_func, K: int, device) -> Union[EngineEvaluator, AutogradEvaluator]:
    eng = getattr(log_prob_func, "_vihmc_engine", None)
    if eng is not None:
        return EngineEvaluator(eng)
    return AutogradEvaluator(log_prob_func, K, device)


# ------------------------------------------------------------------------------------------------
# random streams
# ------------------------------------------------------------------------------------------------
class ChainRNG:
    """Momentum (standard normal [C, K]) and log-uniform [C] draws, in hamiltorch's call order."""

    def __init__(self, C: int, K: int, device, seeds: Optional[Sequence[int]] = None, mode: str = "per_chain"):
        self.C, self.K, self.device, self.mode = C, K, torch.device(device), mode
        if mode == "global":
            if C != 1:
                raise ValueError("rng='global' reproduces hamiltorch's single-chain global-generator stream; C must be 1")
        elif mode == "per_chain":
            if seeds is None or len(seeds) != C:
                raise ValueError("rng='per_chain' needs one seed per chain")
            self.gens = [torch.Generator().manual_seed(int(s)) for s in seeds]
            self._zeros = torch.zeros(K)
            self._ones = torch.ones(K)
        else:
            raise ValueError(f"unknown rng mode {mode!r}")
        self._pin = self.device.type == "cuda"
        self._ahead = None             # (generator states before the draw, momenta) of prefetch_momentum

    def prefetch_momentum(self):
        """Draw the NEXT draw_momentum()'s momenta now (the runner does this while the device works). Transparent to
        every other use of this object: the generators' states before the draw are kept, and any other draw that
        comes first rewinds them and drops the prefetch, so each chain's stream keeps hamiltorch's call order whoever
        else draws from it."""
        if self.mode != "per_chain" or self._ahead is not None:
            return
        states = [g.get_state() for g in self.gens]
        self._ahead = (states, self._draw_momentum())

    def _rewind(self):
        if self._ahead is not None:
            for g, st in zip(self.gens, self._ahead[0]):
                g.set_state(st)
            self._ahead = None

    def draw_momentum(self) -> torch.Tensor:
        """Standard-normal momenta [C, K] on the device (hamiltorch gibbs)."""
        if self._ahead is not None:
            z = self._ahead[1]
            self._ahead = None
            return z
        return self._draw_momentum()

    def _draw_momentum(self) -> torch.Tensor:
        if self.mode == "global":
            return torch.normal(torch.zeros(self.K, device=self.device), torch.ones(self.K, device=self.device))[None]
        z = torch.empty(self.C, self.K, pin_memory=self._pin)
        for c, g in enumerate(self.gens):
            torch.normal(self._zeros, self._ones, generator=g, out=z[c])
        return z.to(self.device, non_blocking=True)

    def draw_logu(self, mask=None) -> torch.Tensor:
        """log(torch.rand(1)) per chain on the device (hamiltorch's accept draw, computed on the CPU);
        chains with mask[c] False do not consume their stream (value -inf)."""
        self._rewind()
        if self.mode == "global":
            if mask is not None and not mask[0]:        # hamiltorch raised LogProbError: no draw
                return torch.full((1,), float("-inf"), device=self.device)
            return torch.log(torch.rand(1)).to(self.device)
        lu = torch.full((self.C,), float("-inf"), pin_memory=self._pin)
        for c, g in enumerate(self.gens):
            if mask is None or mask[c]:
                lu[c] = torch.log(torch.rand(1, generator=g))[0]
        return lu.to(self.device, non_blocking=True)

    def draw(self):
        z = self.draw_momentum()
        return z, self.draw_logu()


# ------------------------------------------------------------------------------------------------
# dual averaging (hamiltorch adaptation, host arithmetic per chain)
# ------------------------------------------------------------------------------------------------
def adaptation(rho, t, step_size_init, H_t, eps_bar, desired_accept_rate=0.8):
    t = t + 1
    r = torch.tensor([rho])
    if bool(torch.isnan(r).any()) or bool(torch.isinf(r).any()):
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


# ------------------------------------------------------------------------------------------------
# batched chains
# ------------------------------------------------------------------------------------------------
@dataclass
class ChainResult:
    samples: torch.Tensor          # [C, S_cap, K] (rows >= counts[c] are unused)
    counts: torch.Tensor           # [C] number of stored samples per chain (hamiltorch's len(ret_params))
    accepted: torch.Tensor         # [C, num_samples] bool
    logp_trace: torch.Tensor       # [C, num_samples] log-prob of the chain state after each iteration
    step_size: List[float]         # final step size per chain
    n_grad_evals: int = 0          # chain-gradient evaluations actually performed
    n_value_evals: int = 0
    extra: dict = field(default_factory=dict)

    def chain(self, c: int) -> List[torch.Tensor]:
        """hamiltorch's return format for chain c: a list of [K] tensors."""
        return list(self.samples[c, :int(self.counts[c])].unbind(0))

    def stacked(self) -> torch.Tensor:
        """[C, S, K] when every chain stored the same number of samples."""
        n = int(self.counts.min())
        if int(self.counts.max()) != n:
            raise RuntimeError("chains stored different numbers of samples (LogProbError rejections)")
        return self.samples[:, :n]


def _grad(ev, theta):
    """gradient-only evaluation of an inner leapfrog step (hamiltorch discards its log-prob); evaluators without
    ``grad`` (any object with the logp_grad / logp contract) fall back to logp_grad"""
    f = getattr(ev, "grad", None)
    return f(theta) if f is not None else ev.logp_grad(theta)[1]


def _kinetic(p, inv_mass):
    return 0.5 * (p * p).sum(1) if inv_mass is None else 0.5 * (p * (inv_mass * p)).sum(1)


class HMCRunner:
    """C independent chains from theta0 [C, K], advanced one HMC iteration per ``step()``.

    ``evaluators`` is one evaluator, or a list of per-shard evaluators for ``Integrator.SPLITTING``
    (each closure already divides its prior by prior_scale, as define_split_model_log_prob does).

    RNG order: hamiltorch draws the accept uniform only when both Hamiltonians are finite (a
    ``LogProbError`` skips it). ``strict_rng=True`` reproduces that exactly at the price of one host
    synchronisation per sample; the default draws every chain's uniform up front (identical streams
    whenever no log-prob is non-finite) so the whole iteration stays on the device.
    """

    def __init__(self, evaluators, theta0: torch.Tensor, num_samples: int, num_steps_per_sample: int, step_size,
                 burn: int = 0, inv_mass: Optional[torch.Tensor] = None, sampler: Sampler = Sampler.HMC,
                 integrator: Integrator = Integrator.IMPLICIT, desired_accept_rate: float = 0.8,
                 rng: Optional[ChainRNG] = None, seeds: Optional[Sequence[int]] = None,
                 reuse_endpoint_grad: bool = True, store: bool = True, strict_rng: bool = False):
        evs = list(evaluators) if isinstance(evaluators, (list, tuple)) else [evaluators]
        self.splitting = integrator == Integrator.SPLITTING
        if self.splitting and len(evs) < 2:
            raise RuntimeError("For splitting log_prob_func must be list of functions")
        if not self.splitting and len(evs) != 1:
            raise RuntimeError("a list of log_prob_funcs needs Integrator.SPLITTING")
        if sampler == Sampler.RMHMC:
            raise NotImplementedError("RMHMC is not on the VI-HMC path (no reference call site)")
        if burn >= num_samples:
            raise RuntimeError("burn must be less than num_samples.")
        self.nuts = sampler == Sampler.HMC_NUTS
        if self.nuts and burn == 0:
            raise RuntimeError("burn must be greater than 0 for NUTS.")
        self.evs = evs
        self.device = device = evs[0].device
        theta = theta0.to(device=device, dtype=torch.float32).contiguous().clone()
        if theta.dim() == 1:
            theta = theta[None]
        self.C, self.K = C, K = theta.shape
        self.rng = rng if rng is not None else ChainRNG(C, K, device, seeds if seeds is not None else list(range(C)))
        self.L, self.M = int(num_steps_per_sample), len(evs)
        self.num_samples, self.burn = num_samples, burn
        self.reuse, self.store, self.strict = reuse_endpoint_grad, store, strict_rng
        self.desired_accept_rate = desired_accept_rate
        self.inv_mass = self.mass_sqrt = None
        if inv_mass is not None:
            self.inv_mass = inv_mass.to(device=device, dtype=torch.float32)
            if self.inv_mass.dim() != 1:
                raise NotImplementedError("only a diagonal (1-D) inv_mass is supported on the batched path")
            self.mass_sqrt = (1 / self.inv_mass) ** 0.5
        # step sizes: python float (bitwise hamiltorch) or per-chain fp32 column under NUTS adaptation
        self.eps_host = [float(step_size)] * C
        self.step_size_init = float(step_size)
        self.H_t = [0.0] * C
        self.eps_bar = [1.0] * C
        # initial state: logp (sum over shards) and the shard-0 gradient that opens a trajectory
        lp0, g0 = evs[0].logp_grad(theta)
        for m in range(1, self.M):
            lp0 = lp0 + evs[m].logp(theta)
        self.cur = [theta, lp0, g0]
        self.last_ret = [t.clone() for t in self.cur]
        self.burn_prev = [t.clone() for t in self.cur]
        S_cap = num_samples + 2 if store else 2
        self.samples = torch.empty(C, S_cap, K, device=device)
        self.samples[:, 0] = theta
        self.counts = torch.ones(C, dtype=torch.long, device=device)
        self.accepted = torch.zeros(C, num_samples, dtype=torch.bool, device=device)
        self.trace = torch.empty(C, num_samples, device=device)
        # the Metropolis step on the GPU in one launch (vihmc_hmc_accept) instead of ~30 small torch ops per
        # iteration; the torch form below stays for CPU chains and strict_rng (whose accept draw needs ok first)
        # (engine evaluators only: a runner over user torch closures never needs libvihmc)
        self._accept_native = (device.type == "cuda" and not self.strict
                               and all(isinstance(e, EngineEvaluator) for e in self.evs))
        self._rows = torch.arange(C, device=device) * S_cap
        self.n = 0
        # kinetic energies in one vihmc_kinetic launch (engine evaluators on CUDA; both accept forms use it, so they
        # stay bitwise equal) instead of 0.5 * (p * p).sum(1)'s four; its workspace is zeroed once here
        # strict_rng (the hamiltorch drop-in sample()) keeps the reference's fp32 0.5 * (p * p).sum(): accept decisions
        # within a few ulps of the margin then fall as hamiltorch's do
        self._native_ke = (device.type == "cuda" and not self.strict
                           and all(isinstance(e, EngineEvaluator) for e in self.evs))
        self._ke_ws = None

    def _ke(self, p):
        """The kinetic energy of every chain [C] (hamiltorch's 0.5 p.p, or 0.5 p.(inv_mass p))."""
        if not self._native_ke:
            return _kinetic(p, self.inv_mass)
        import ctypes
        from . import _lib
        L = _lib.lib()
        C, K = p.shape
        if self._ke_ws is None:
            S = int(L.vihmc_kinetic_slices(K))
            self._ke_ws = (torch.zeros(C * S, dtype=torch.float64, device=self.device),
                           torch.zeros(C, dtype=torch.int32, device=self.device))
        part, cnt = self._ke_ws
        p = p.to(torch.float32).contiguous()
        im = None if self.inv_mass is None else self.inv_mass.to(torch.float32).contiguous()
        ke = torch.empty(C, device=self.device)

        def ptr(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None
        with torch.cuda.device(self.device):
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
            _lib.check(L.vihmc_kinetic(ptr(p), ptr(im), C, K, ptr(ke), ptr(part), ptr(cnt), stream), "vihmc_kinetic")
        return ke

    def _eps(self):
        if not self.nuts:
            return self.eps_host[0]
        return torch.tensor(self.eps_host, dtype=torch.float32, device=self.device)[:, None]

    def _trajectory(self, th, g, p, eps):
        evs, L, M, inv_mass = self.evs, self.L, self.M, self.inv_mass
        if not self.splitting and getattr(evs[0], "fused_trajectory", False):
            g_open = g if self.reuse else evs[0].logp_grad(th)[1]
            th, p, lp_new, g_new = evs[0].trajectory(th, p, g_open, eps if not torch.is_tensor(eps) else eps[:, 0],
                                                     L, inv_mass)
            return th, p, lp_new, g_new
        if not self.splitting:
            g_open = g if self.reuse else evs[0].logp_grad(th)[1]
            p = p + (0.5 * eps) * g_open
            lp_new = g_new = None
            for step in range(L):
                th = th + eps * p if inv_mass is None else th + eps * inv_mass * p
                if step == L - 1:
                    lp_new, g_new = evs[0].logp_grad(th)
                else:
                    g_new = _grad(evs[0], th)
                p = p + eps * g_new
            p = p - (0.5 * eps) * g_new
            return th, p, lp_new, g_new
        sub = eps / (2 * (M - 1))
        if self._fused_split(eps):
            return self._trajectory_split_fused(th, g, p, eps)
        g0_cached = g if self.reuse else None
        gm = lp0_end = None
        # one fused kernel per update (torch.add with alpha; eps is a host float here) instead of a scale and
        # an add: config 4's per-step updates between the engine evaluations are launch-bound
        half = 0.5 * eps
        for step in range(L):
            for m in range(M):
                if m == 0 and g0_cached is not None:
                    gm = g0_cached
                elif step == 0 and m == 0:
                    # the trajectory's start point: the residual form, as at its end point (time-symmetric form
                    # assignment), also without the reuse
                    gm = evs[m].logp_grad(th)[1]
                else:
                    gm = _grad(evs[m], th)
                p = torch.add(p, gm, alpha=half) if not torch.is_tensor(eps) else p + half * gm
                if m < M - 1:
                    th = torch.add(th, p, alpha=sub) if not torch.is_tensor(eps) else th + sub * p
            for m in reversed(range(M)):
                if not (m == M - 1 and self.reuse):      # same theta as the forward pass' last shard
                    if step == L - 1 and m == 0:         # only the end point's log-prob is used
                        lp0_end, gm = evs[m].logp_grad(th)
                    else:
                        gm = _grad(evs[m], th)
                p = torch.add(p, gm, alpha=half) if not torch.is_tensor(eps) else p + half * gm
                if m > 0:
                    th = torch.add(th, p, alpha=sub) if not torch.is_tensor(eps) else th + sub * p
            g0_cached = gm if self.reuse else None
        lp_sum = lp0_end.clone()
        for m in range(1, M):
            lp_sum = lp_sum + evs[m].logp(th)
        return th, p, lp_sum, gm

    def _fused_split(self, eps) -> bool:
        """The splitting trajectory with its updates inside the engines' gradient gathers (vihmc_split_step): two
        DeepONet shards, the reused end gradient, a scalar step, no mass matrix (the torch path's own restrictions
        for the updates it fuses); engine attribute ``fused_split = False`` turns it off."""
        if not (self.splitting and self.M == 2 and self.reuse and self.inv_mass is None and not torch.is_tensor(eps)):
            return False
        if self.device.type != "cuda" or not all(isinstance(e, EngineEvaluator) for e in self.evs):
            return False
        from .engine import DeepONetEngine
        return all(isinstance(e.engine, DeepONetEngine) and getattr(e.engine, "fused_split", True)
                   and e.engine._sample_rng is None for e in self.evs)

    def _trajectory_split_fused(self, th, g, p, eps):
        """HMCRunner._trajectory's splitting branch for M = 2 with reuse, the kicks and drifts applied by the
        evaluations' gradient gathers. The loop body there, per step: [m = 0] p += h g0; th += s p; [m = 1] g1 at th;
        p += h g1; (reverse) [m = 1, reused] p += h g1; th += s p; [m = 0] g0 at th; p += h g0. The opening
        p += h g; th += s p stays two torch.add; then every shard-1 evaluation applies its two kicks and the drift
        (mode 1) and writes the new position into shard 0's weights, and every shard-0 evaluation applies its kick,
        the next step's kick and the drift into shard 1 (mode 1), the last one only its kick (mode 2) -- the same
        fma per update as torch.add(alpha=), so bitwise the torch-op path."""
        ev0, ev1 = self.evs
        e0, e1 = ev0.engine, ev1.engine
        L, C = self.L, th.shape[0]
        half = 0.5 * eps
        sub = eps / 2
        p = torch.add(p, g, alpha=half)
        th = torch.add(th, p, alpha=sub)                 # new tensors: the caller's state stays for a rejection
        lp0_end = g0 = None
        for step in range(L):
            ev1.n_grad += C
            e1.split_step(th, p, 1, half, sub, scatter_into=e0, scattered_in=step > 0)
            ev0.n_grad += C
            if step == L - 1:
                lp0_end, g0 = e0.split_step(th, p, 2, half, want_logp=True, scattered_in=True)
            else:
                _, g0 = e0.split_step(th, p, 1, half, sub, scatter_into=e1, scattered_in=True)
        lp_sum = lp0_end + ev1.logp(th)
        return th, p, lp_sum, g0

    def step(self):
        """One HMC iteration for every chain (hamiltorch ``sample`` loop body)."""
        n = self.n
        if n >= self.num_samples:
            raise RuntimeError("all samples drawn")
        rng = self.rng
        z = rng.draw_momentum()                 # prefetched by _draw_ahead at the end of the previous iteration
        logu = None if self.strict else rng.draw_logu()
        p = z if self.mass_sqrt is None else z * self.mass_sqrt
        th, lp, g = self.cur
        if self._accept_native:
            ke0 = self._ke(p)
            th_new, p, lp_new, g_new = self._trajectory(th, g, p, self._eps())
            rho, err = self._accept_fused(n, lp, ke0, th_new, self._ke(p), lp_new, g_new, logu)
            self._draw_ahead(n)
            self._adapt(n, rho, err)
            self.n += 1
            return
        H0 = -lp + self._ke(p)
        th_new, p, lp_new, g_new = self._trajectory(th, g, p, self._eps())
        H1 = -lp_new + self._ke(p)
        d = H0 - H1
        rho = torch.where(torch.isnan(d), torch.zeros_like(d), torch.clamp(d, max=0.0))
        ok = torch.isfinite(lp) & torch.isfinite(lp_new)
        if self.strict:
            logu = rng.draw_logu(ok.tolist())                      # host sync: hamiltorch skips the draw on error
        acc = ok & (rho >= logu)
        err = ~ok
        new = [th_new, lp_new, g_new]

        def sel(mask, a, b):
            return torch.where(mask[:, None] if a.dim() == 2 else mask, a, b)

        if n > self.burn:
            nxt = [sel(acc, nw, lr) for nw, lr in zip(new, self.last_ret)]
            self.last_ret = nxt
            if self.store:
                valid = ~err
                row = torch.where(valid, self.counts, torch.full_like(self.counts, self.samples.shape[1] - 1))
                self.samples.view(-1, self.K).index_copy_(0, self._rows + row, nxt[0])
                self.counts = self.counts + valid.long()
        else:
            fallback = [sel(err, lr, bp) for lr, bp in zip(self.last_ret, self.burn_prev)]
            nxt = [sel(acc, nw, fb) for nw, fb in zip(new, fallback)]
            self.burn_prev = [sel(acc, nw, bp) for nw, bp in zip(new, self.burn_prev)]
        self.cur = nxt
        self.accepted[:, n] = acc
        self.trace[:, n] = nxt[1]
        self._draw_ahead(n)
        self._adapt(n, torch.where(err, torch.full_like(rho, float("nan")), rho), err)
        self.n += 1

    def _draw_ahead(self, n):
        """Iteration n + 1's momenta, drawn on the host now -- after iteration n's last draw (its accept uniform), so
        each chain's stream keeps hamiltorch's order -- while iteration n runs on the device: config 4's 172,401 CPU
        normals per chain otherwise left the GPU idle ~0.33 ms per iteration (profiles/r05lt_c1_trace.txt). The
        prefetch lives in the ChainRNG, which rewinds it if anything else draws first, so a caller-supplied generator
        shared with other code keeps hamiltorch's order; only when an iteration n + 1 exists."""
        if self.rng.mode == "per_chain" and self.device.type == "cuda" and n + 1 < self.num_samples:
            self.rng.prefetch_momentum()

    def _accept_fused(self, n, lp, ke0, th_new, ke1, lp_new, g_new, logu):
        """The accept block above for CUDA chains in one vihmc_hmc_accept launch (the same kinetic energies and
        selection, bit for bit). After burn-in the last returned state is updated in place and is the current
        state."""
        import ctypes
        from . import _lib
        L = _lib.lib()
        C, K = self.C, self.K
        burn = n <= self.burn

        def ptr(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        f32 = [lp, ke0, th_new, ke1, lp_new, g_new, logu]
        lp, ke0, th_new, ke1, lp_new, g_new, logu = [t.to(torch.float32).contiguous() for t in f32]
        rho = torch.empty(C, device=self.device)
        err = torch.empty(C, dtype=torch.uint8, device=self.device)
        last = self.last_ret
        if burn:
            cur = [torch.empty_like(t) for t in last]
            bp = self.burn_prev
        else:
            cur = last
            bp = [None, None, None]
        samples = self.samples if (self.store and not burn) else None
        with torch.cuda.device(self.device):
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
            rc = L.vihmc_hmc_accept(C, K, n, 1 if burn else 0, ptr(lp), ptr(lp_new), ptr(ke0), ptr(ke1),
                                  ptr(logu), ptr(th_new), ptr(g_new),
                                  ptr(last[0]), ptr(last[1]), ptr(last[2]), ptr(bp[0]), ptr(bp[1]), ptr(bp[2]),
                                  ptr(cur[0]) if burn else None, ptr(cur[1]) if burn else None,
                                  ptr(cur[2]) if burn else None, ptr(samples), self.samples.shape[1],
                                  ptr(self.counts), ptr(self.accepted), self.accepted.stride(0), ptr(self.trace),
                                  self.trace.stride(0), ptr(rho), ptr(err), stream)
        _lib.check(rc, "vihmc_hmc_accept")
        self.cur = cur
        return rho, err.bool()

    def _adapt(self, n, rho, err):
        """NUTS dual averaging of every chain's step size during burn-in (rho: NaN where the chain failed)."""
        if self.nuts and n <= self.burn:
            rho_h = rho.tolist()                                   # host sync (burn only)
            err_h = err.tolist()
            for c in range(self.C):
                if n < self.burn or err_h[c]:
                    self.eps_host[c], self.eps_bar[c], self.H_t[c] = adaptation(
                        rho_h[c], n, self.step_size_init, self.H_t[c], self.eps_bar[c], self.desired_accept_rate)
                if n == self.burn:
                    self.eps_host[c] = self.eps_bar[c]

    def result(self) -> ChainResult:
        return ChainResult(self.samples, self.counts, self.accepted[:, :self.n], self.trace[:, :self.n],
                           list(self.eps_host), sum(e.n_grad for e in self.evs), sum(e.n_value for e in self.evs))


def run_chains(evaluators, theta0: torch.Tensor, num_samples: int, num_steps_per_sample: int, step_size,
               **kw) -> ChainResult:
    """Run C independent chains for ``num_samples`` iterations (see HMCRunner)."""
    r = HMCRunner(evaluators, theta0, num_samples, num_steps_per_sample, step_size, **kw)
    for _ in range(num_samples):
        r.step()
    return r.result()


# ------------------------------------------------------------------------------------------------
# hamiltorch-compatible entry point
# ------------------------------------------------------------------------------------------------
def sample(log_prob_func, params_init, num_samples=10, num_steps_per_sample=10, step_size=0.1, burn=0, jitter=None,
           inv_mass=None, normalizing_const=1., softabs_const=None, explicit_binding_const=100,
           fixed_point_threshold=1e-5, fixed_point_max_iterations=1000, jitter_max_tries=10, sampler=Sampler.HMC,
           integrator=Integrator.IMPLICIT, metric=None, debug=False, desired_accept_rate=0.8, store_on_GPU=True,
           pass_grad=None, verbose=False, rng: str = "global", seed: Optional[int] = None):
    """Drop-in for ``hamiltorch.samplers.sample`` on the VI-HMC path: returns a list of [K] tensors
    (hamiltorch's ``ret_params``). A ``log_prob_func`` built by vihmc's ``define_model_log_prob`` runs
    on the batched HIP engine; any other torch closure runs through autograd. ``debug=2`` returns
    (samples, acceptance rate) / (samples, step size) for NUTS as hamiltorch does."""
    if params_init.dim() != 1:
        raise RuntimeError("params_init must be a 1d tensor.")
    fns = log_prob_func if isinstance(log_prob_func, list) else [log_prob_func]
    K = params_init.shape[0]
    device = params_init.device
    evs = [evaluator_for(f, K, device) for f in fns]
    device = evs[0].device
    if rng == "global":
        r = ChainRNG(1, K, device, mode="global")
    else:
        r = ChainRNG(1, K, device, seeds=[seed if seed is not None else torch.initial_seed()])
    # strict_rng: a non-finite log-prob skips the accept draw exactly as hamiltorch's LogProbError does (one
    # host sync per sample; hamiltorch syncs on every accept anyway)
    res = run_chains(evs if len(evs) > 1 else evs[0], params_init[None], num_samples, num_steps_per_sample, step_size,
                     burn=burn, inv_mass=inv_mass, sampler=sampler, integrator=integrator,
                     desired_accept_rate=desired_accept_rate, rng=r, strict_rng=True)
    out = [t.to(params_init.device) for t in res.chain(0)]
    if not verbose:
        rate = 1 - float((~res.accepted[0]).sum()) / num_samples
        print(f"Acceptance Rate {rate:.2f}")
    if debug == 2:
        if sampler == Sampler.HMC_NUTS:
            return out, res.step_size[0]
        return out, 1 - float((~res.accepted[0]).sum()) / num_samples
    return out

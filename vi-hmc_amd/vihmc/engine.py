"""Batched log-posterior + gradient engines over libvihmc.so plans.

These are the MI355X replacement of the reference's ``log_prob_func`` + ``torch.autograd.grad``
pair (Operator_network/VI_HMC/main_VI_HMC_burgers.py:86-178; Neural_network/VI_HMC/
main_VI_HMC.py:96-151): one call evaluates C chains, theta [C, K] -> (logp [C], grad [C, K]), all
device-resident, enqueued on torch's current HIP stream with no host synchronisation.
"""
from __future__ import annotations

import ctypes
import random
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from .layout import DeepONetSpec, MLPSpec

LOSS_CODES = {"NLL": 0, "regression": 1}


def _c32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _linears(layers) -> ctypes.Array:
    arr = (_lib.Linear * len(layers))()
    for i, l in enumerate(layers):
        arr[i].w_off, arr[i].b_off, arr[i].n_out, arr[i].n_in, arr[i].act = l.w_off, l.b_off, l.n_out, l.n_in, l.act
    return arr


def _lik(loss: str, tau_out: float, prior_scale: float) -> _lib.LikDesc:
    if loss not in LOSS_CODES:
        raise NotImplementedError(f"loss {loss!r}: the hot path implements 'NLL' and 'regression'")
    return _lib.LikDesc(LOSS_CODES[loss], float(tau_out), float(prior_scale), 0)


class _Engine:
    kind = "?"

    def __init__(self, device):
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("vihmc engines run on a HIP device (torch 'cuda'); there is no CPU fallback")
        if not torch.cuda.is_available():
            raise RuntimeError("no HIP device visible: the vihmc engine has no CPU fallback")
        self.device = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
        self._plan = ctypes.c_void_p()
        self.L = _lib.lib()
        self._sample_rng = None               # cfg.sample_data: redraw the trunk rows before each evaluation

    # ---- plan lifetime ---------------------------------------------------------------------------
    def _created(self, rc, what):
        _lib.check(rc, what)
        self.K = self.L.vihmc_plan_K(self._plan)
        self.D = self.L.vihmc_plan_n_params(self._plan)
        self.max_chains = self.L.vihmc_plan_max_chains(self._plan)
        self.device_bytes = self.L.vihmc_plan_device_bytes(self._plan)

    def close(self):
        if getattr(self, "_plan", None) is not None and self._plan.value:
            self.L.vihmc_plan_destroy(self._plan)
            self._plan = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- evaluation ------------------------------------------------------------------------------
    def _theta(self, theta: torch.Tensor) -> torch.Tensor:
        if theta.dim() == 1:
            theta = theta.unsqueeze(0)
        if theta.dim() != 2 or theta.shape[1] != self.K:
            raise ValueError(f"theta must be [C, {self.K}] (got {tuple(theta.shape)})")
        if theta.shape[0] > self.max_chains:
            raise ValueError(f"C={theta.shape[0]} exceeds the plan's max_chains={self.max_chains}")
        return theta.to(device=self.device, dtype=torch.float32).contiguous()

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def logp_grad(self, theta: torch.Tensor, logp: Optional[torch.Tensor] = None,
                  grad: Optional[torch.Tensor] = None):
        """theta [C, K] -> (logp [C], grad [C, K]) on the engine's device."""
        th = self._theta(theta)
        if self._sample_rng is not None:
            self._redraw()
        C = th.shape[0]
        if logp is None:
            logp = torch.empty(C, device=self.device, dtype=torch.float32)
        if grad is None:
            grad = torch.empty(C, self.K, device=self.device, dtype=torch.float32)
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_logp_grad(self._plan, th.data_ptr(), C, logp.data_ptr(), grad.data_ptr(), self._stream())
        _lib.check(rc, "vihmc_logp_grad")
        return logp, grad

    def grad(self, theta: torch.Tensor, grad: Optional[torch.Tensor] = None) -> torch.Tensor:
        """theta [C, K] -> grad [C, K] only (vihmc_grad: the leapfrog's inner evaluations; DeepONet plans run the
        Gram-form contraction there)."""
        th = self._theta(theta)
        if self._sample_rng is not None:
            self._redraw()
        C = th.shape[0]
        if grad is None:
            grad = torch.empty(C, self.K, device=self.device, dtype=torch.float32)
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_grad(self._plan, th.data_ptr(), C, grad.data_ptr(), self._stream())
        _lib.check(rc, "vihmc_grad")
        return grad

    def logp(self, theta: torch.Tensor, logp: Optional[torch.Tensor] = None) -> torch.Tensor:
        th = self._theta(theta)
        if self._sample_rng is not None:
            self._redraw()
        C = th.shape[0]
        if logp is None:
            logp = torch.empty(C, device=self.device, dtype=torch.float32)
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_logp_grad(self._plan, th.data_ptr(), C, logp.data_ptr(), None, self._stream())
        _lib.check(rc, "vihmc_logp_grad(value)")
        return logp

    def forward(self, theta: torch.Tensor):
        """theta [C, K] -> (logp [C], network output [C, *out_shape])."""
        th = self._theta(theta)
        C = th.shape[0]
        logp = torch.empty(C, device=self.device, dtype=torch.float32)
        out = torch.empty((C,) + tuple(self.out_shape), device=self.device, dtype=torch.float32)
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_forward(self._plan, th.data_ptr(), C, logp.data_ptr(), out.data_ptr(), self._stream())
        _lib.check(rc, "vihmc_forward")
        return logp, out

    def trajectory(self, theta: torch.Tensor, momentum: torch.Tensor, grad: torch.Tensor, eps, L: int,
                   inv_mass: Optional[torch.Tensor] = None):
        """One whole leapfrog trajectory of every chain (vihmc_trajectory: one launch for BNN plans; for DeepONet
        plans L evaluations with the momentum / position steps fused into their gradient gather): from theta
        [C, K], the fresh momentum and the gradient at theta, L steps of size eps (python float or per-chain [C])
        -> (theta_L, p_L, logp_L, grad_L), bitwise the step-by-step path."""
        if self._sample_rng is not None:
            raise RuntimeError("cfg.sample_data redraws the trunk rows per evaluation: use the step-by-step path")
        th = self._theta(theta)
        C = th.shape[0]
        p = momentum.to(self.device, torch.float32).contiguous()
        g = grad.to(self.device, torch.float32).contiguous()
        if p.shape != th.shape or g.shape != th.shape:
            raise ValueError("momentum and grad must match theta [C, K]")
        e = (torch.full((C,), float(eps), dtype=torch.float32, device=self.device) if not torch.is_tensor(eps)
             else eps.to(self.device, torch.float32).reshape(-1).expand(C).contiguous())
        im = None if inv_mass is None else inv_mass.to(self.device, torch.float32).reshape(-1).contiguous()
        if im is not None and im.numel() != self.K:
            raise ValueError(f"inv_mass must be [{self.K}]")
        th_out, p_out, g_out = torch.empty_like(th), torch.empty_like(th), torch.empty_like(th)
        lp = torch.empty(C, device=self.device, dtype=torch.float32)
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_trajectory(self._plan, th.data_ptr(), th_out.data_ptr(), p.data_ptr(), p_out.data_ptr(),
                                         g.data_ptr(), g_out.data_ptr(), lp.data_ptr(), e.data_ptr(),
                                         None if im is None else im.data_ptr(), int(L), C, self._stream())
        _lib.check(rc, "vihmc_trajectory")
        return th_out, p_out, lp, g_out

    def split_step(self, theta: torch.Tensor, momentum: torch.Tensor, mode: int, kick: float, drift: float = 0.0,
                   scatter_into=None, scattered_in: bool = False, want_logp: bool = False):
        """vihmc_split_step: this shard's gradient at theta [C, K] (a float32 device tensor updated IN PLACE, as is
        momentum) with the splitting integrator's updates around it applied by the gradient gather -- mode 1:
        p += kick g twice, then theta += drift p, scattered into `scatter_into`'s weights (the next shard's engine);
        mode 2: p += kick g. Returns (logp or None, grad). Bitwise the torch.add(alpha=) sequence of
        HMCRunner._trajectory's splitting branch."""
        if self._sample_rng is not None:
            raise RuntimeError("cfg.sample_data redraws the trunk rows per evaluation: use the step-by-step path")
        if (theta.dtype != torch.float32 or not theta.is_contiguous() or theta.device != self.device
                or tuple(theta.shape[1:]) != (self.K,)):
            raise ValueError("theta must be a contiguous float32 [C, K] tensor on the plan's device (updated in place)")
        if momentum.shape != theta.shape or momentum.dtype != torch.float32 or not momentum.is_contiguous() \
                or momentum.device != self.device:
            raise ValueError("momentum must match theta (contiguous float32, same device; updated in place)")
        C = theta.shape[0]
        grad = torch.empty(C, self.K, device=self.device, dtype=torch.float32)
        lp = torch.empty(C, device=self.device, dtype=torch.float32) if want_logp else None
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_split_step(self._plan, theta.data_ptr(), momentum.data_ptr(), C, grad.data_ptr(),
                                         None if lp is None else lp.data_ptr(), int(mode), float(kick), float(drift),
                                         None if scatter_into is None else scatter_into._plan, int(bool(scattered_in)),
                                         self._stream())
        _lib.check(rc, "vihmc_split_step")
        return lp, grad

    def set_data(self, x_branch: torch.Tensor, y: torch.Tensor):
        """vihmc_plan_set_data (DeepONet): new branch rows [N, in_branch] and targets [N, P], same N / P."""
        xb = torch.as_tensor(x_branch).to(device=self.device, dtype=torch.float32).contiguous()
        yy = torch.as_tensor(y).to(device=self.device, dtype=torch.float32).contiguous()
        if xb.numel() != self.N * self.spec.in_branch or yy.numel() != self.N * self.P:
            raise ValueError(f"set_data needs x_branch [{self.N}, {self.spec.in_branch}] and y [{self.N}, {self.P}]")
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_plan_set_data(self._plan, xb.data_ptr(), yy.data_ptr(), self._stream())
        _lib.check(rc, "vihmc_plan_set_data")
        self._keep_data = (xb, yy)          # the copy is asynchronous on the stream

    def set_sample_grid(self, trunk_feat_all: torch.Tensor, y_all: torch.Tensor):
        """The full trunk grid cfg.sample_data draws from (main_VI_HMC_burgers.py:131-134): trunk features
        [P_all, in_trunk] (as the plan was built with, i.e. after any feature map) and targets [N, P_all],
        kept resident on the device; select rows with set_trunk_rows."""
        ft = torch.as_tensor(trunk_feat_all).to(device=self.device, dtype=torch.float32).contiguous()
        ya = torch.as_tensor(y_all).to(device=self.device, dtype=torch.float32).contiguous()
        if ft.dim() != 2 or ft.shape[1] != self.spec.in_trunk or ya.shape != (self.N, ft.shape[0]):
            raise ValueError(f"set_sample_grid needs trunk features [P_all, {self.spec.in_trunk}] and y "
                             f"[{self.N}, P_all]")
        if ft.shape[0] < self.P:
            raise ValueError(f"the grid has {ft.shape[0]} rows < the plan's P={self.P}")
        self._grid = (ft, ya)

    def set_trunk_rows(self, ind):
        """vihmc_plan_set_trunk_rows: evaluate at grid rows ``ind`` ([P] ints in [0, P_all)) from now on."""
        if getattr(self, "_grid", None) is None:
            raise RuntimeError("set_trunk_rows needs set_sample_grid first")
        ft, ya = self._grid
        ii = np.asarray(ind, dtype=np.int64).reshape(-1)
        if ii.size != self.P or (ii.size and (ii.min() < 0 or ii.max() >= ft.shape[0])):
            raise ValueError(f"set_trunk_rows needs {self.P} indices in [0, {ft.shape[0]})")
        it = torch.from_numpy(ii.astype(np.int32)).to(self.device)
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_plan_set_trunk_rows(self._plan, ft.data_ptr(), ya.data_ptr(), int(ft.shape[0]),
                                                  it.data_ptr(), self._stream())
        _lib.check(rc, "vihmc_plan_set_trunk_rows")
        self._keep_ind = it                   # the gather is asynchronous on the stream

    def sample_data(self, trunk_feat_all, y_all, p: int, rng=None):
        """cfg.sample_data (main_VI_HMC_burgers.py:131-134): before every logp / logp_grad call draw
        ``rng.sample(range(P_all), p)`` (default: Python's global ``random``, which the reference's
        ``from random import sample`` uses) and evaluate at those trunk rows. One draw per call, shared by the
        C chains of a batched call (the reference's per-chain calls draw once each: identical at C = 1).
        Disables the fused trajectory (it would keep one draw for L steps). ``p=None`` switches it off."""
        if p is None:
            self._sample_rng, self._grid = None, None
            self.fused_trajectory = True
            return
        if int(p) != self.P:
            raise ValueError(f"the plan was built for P={self.P} trunk rows, cfg.p={p}")
        self.set_sample_grid(trunk_feat_all, y_all)
        self._sample_rng = random if rng is None else rng
        self.fused_trajectory = False

    def _redraw(self):
        self.set_trunk_rows(self._sample_rng.sample(range(int(self._grid[0].shape[0])), self.P))

    def sensitivity(self, theta: torch.Tensor, pts=None, sigma=None) -> torch.Tensor:
        """vihmc_sensitivity: sigma^2 * mean over outputs of (d f / d theta)^2 for all D parameters, flat
        order, at theta ([K], the plan's chain 0). DeepONet: ``pts`` [N, npts] int, the trunk points each
        branch row is evaluated at (required); BNN: every data row. ``sigma=None`` returns the mean
        squared gradient."""
        th = self._theta(torch.as_tensor(theta).reshape(1, -1))
        out = torch.empty(self.D, device=self.device, dtype=torch.float32)
        sg = None
        if sigma is not None:
            sg = torch.as_tensor(sigma).to(device=self.device, dtype=torch.float32).reshape(-1).contiguous()
            if sg.numel() != self.D:
                raise ValueError(f"sigma must have D={self.D} entries")
        pp, npts = None, 0
        if self.kind == "deeponet":
            if pts is None:
                raise ValueError("DeepONet sensitivity needs pts [N, npts] (trunk points per branch row)")
            pp = np.ascontiguousarray(np.asarray(pts, dtype=np.int32))
            if pp.ndim != 2 or pp.shape[0] != self.N:
                raise ValueError(f"pts must be [N={self.N}, npts]")
            npts = pp.shape[1]
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_sensitivity(self._plan, th.data_ptr(), None if pp is None else pp.ctypes.data, npts,
                                          None if sg is None else sg.data_ptr(), out.data_ptr(), self._stream())
        _lib.check(rc, "vihmc_sensitivity")
        return out

    # ---- kernel timing hook (roofline) -----------------------------------------------------------
    # classes of include/vihmc.h VIHMC_T_*
    T_CONTRACT_A, T_CONTRACT_B, T_BWD, T_FWD, T_EVAL, T_MLP, T_GRAM = range(7)
    T_ALL = -1

    def timing(self, which: int = 0, on: bool = True):
        """Enable / disable HIP-event timing of kernel class ``which`` (-1: all); discards recorded events."""
        _lib.check(self.L.vihmc_timing_enable(self._plan, which, int(on)), "vihmc_timing_enable")

    def timing_class(self, which: int):
        """(total ms, launches) recorded for one class since the last enable / reset (not discarded)."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        _lib.check(self.L.vihmc_timing_read_class(self._plan, which, ctypes.byref(ms), ctypes.byref(n)),
                   "vihmc_timing_read_class")
        return ms.value, n.value

    def timing_reset(self):
        _lib.check(self.L.vihmc_timing_reset(self._plan), "vihmc_timing_reset")

    def graph(self, on: bool = True):
        """hipGraph replay of the gradient evaluation (vihmc_graph_enable)."""
        _lib.check(self.L.vihmc_graph_enable(self._plan, int(on)), "vihmc_graph_enable")

    def option(self, key: str, value: int):
        """vihmc_plan_option: "fwd_bf16x6" / "contract_bf16x6" / "bwd_bf16x6" (the bf16x6 forms, exact 3-way
        splits), "graph", "fwd_wimg" (0: the fp32-MFMA fused forward), "fwd_in0" (0: the input layers in a launch of
        their own instead of the bf16x6 forward's), "img_scatter" (0: the forward's weight images
        split every evaluation instead of kept by the scatter), "fuse_scatter" (0: trajectory evaluations run their
        own scatter)."""
        _lib.check(self.L.vihmc_plan_option(self._plan, key.encode(), int(value)), f"vihmc_plan_option({key})")

    def get_option(self, key: str) -> int:
        """vihmc_plan_get_option: the option's current value."""
        v = ctypes.c_int()
        _lib.check(self.L.vihmc_plan_get_option(self._plan, key.encode(), ctypes.byref(v)),
                   f"vihmc_plan_get_option({key})")
        return v.value

    def check_canaries(self) -> int:
        """vihmc_plan_check_canaries: bytes written past the end of the plan's buffers (plan created with the
        environment VIHMC_CANARY=1); syncs the device."""
        n = ctypes.c_int64()
        _lib.check(self.L.vihmc_plan_check_canaries(self._plan, ctypes.byref(n)), "vihmc_plan_check_canaries")
        return n.value

    def debug_buffer(self, name: str):
        """vihmc_plan_debug_copy: the named internal buffer (all chains) as raw bytes (numpy uint8), or None when the
        plan has not allocated it; syncs the device. Diagnostics only."""
        import numpy as np
        n = ctypes.c_int64()
        _lib.check(self.L.vihmc_plan_debug_copy(self._plan, name.encode(), None, ctypes.byref(n)), "vihmc_plan_debug_copy")
        if n.value == 0:
            return None
        out = np.empty(n.value, dtype=np.uint8)
        _lib.check(self.L.vihmc_plan_debug_copy(self._plan, name.encode(), out.ctypes.data_as(ctypes.c_void_p),
                                                ctypes.byref(n)), "vihmc_plan_debug_copy")
        return out

    def timing_read(self):
        """(total ms, launches) over every recorded class; discards the events."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        _lib.check(self.L.vihmc_timing_read(self._plan, ctypes.byref(ms), ctypes.byref(n)), "vihmc_timing_read")
        return ms.value, n.value


class ShaderClock:
    """Average shader clock over a region of a stream: vihmc_clock_stamp before and after it (256 one-wave workgroups:
    XCD id, HW_ID, s_memtime, s_memrealtime). Each CU's clock is d memtime / d memrealtime x 100 MHz from ITS OWN two
    readings (workgroups paired by (XCD, CU / shader array / engine)); per XCD the median over its paired CUs.
    Readings above the 2,400-MHz maximum are physically impossible: they are rejected and counted, never averaged."""

    WG = 256
    MAX_MHZ = 2400.0

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf = torch.zeros(2, self.WG, 4, dtype=torch.int64, device=self.device)
        self.L = _lib.lib()

    def _stamp(self, i):
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_clock_stamp(self.buf[i].data_ptr(),
                                          ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        _lib.check(rc, "vihmc_clock_stamp")

    def start(self):
        self._stamp(0)

    def stop(self):
        self._stamp(1)

    @staticmethod
    def _cu_key(xcc, hw):
        # HW_ID: wave [3:0], SIMD [5:4], pipe [7:6], CU [11:8], shader array [12], shader engine [15:13]
        return int(xcc), (int(hw) >> 8) & 0xFF

    def per_cu(self) -> dict:
        """{(xcd, cu key): MHz} for every CU stamped in both readings (syncs)."""
        b = self.buf.cpu().numpy().view(np.uint64)
        first = [{}, {}]
        for i in range(2):
            for row in b[i]:
                first[i].setdefault(self._cu_key(row[0], row[1]), (float(row[2]), float(row[3])))
        out = {}
        for k, (t0, r0) in first[0].items():
            if k in first[1]:
                t1, r1 = first[1][k]
                if r1 > r0:
                    out[k] = 100.0 * (t1 - t0) / (r1 - r0)
        return out

    def summary(self) -> dict:
        """Per-XCD medians of the valid per-CU clocks, their spread, and the rejected readings."""
        cu = self.per_cu()
        bad = {f"{k[0]}:{k[1]}": round(v, 1) for k, v in cu.items() if not (0.0 < v <= self.MAX_MHZ)}
        by_xcd = {}
        for (x, _), v in cu.items():
            if 0.0 < v <= self.MAX_MHZ:
                by_xcd.setdefault(x, []).append(v)
        med = {x: float(np.median(v)) for x, v in sorted(by_xcd.items())}
        vals = list(med.values())
        mean = float(np.mean(vals)) if vals else None
        spread = (max(vals) - min(vals)) / mean if vals else None
        return {"mhz_by_xcd": med, "mean_mhz": mean, "spread": spread, "cus_paired": len(cu),
                "cus_per_xcd": {x: len(v) for x, v in sorted(by_xcd.items())}, "rejected_above_max": bad}

    def mhz(self) -> dict:
        """{xcd: MHz}: the per-XCD medians of summary()."""
        return self.summary()["mhz_by_xcd"]


def expand_prior(K: int, mu, sd) -> (np.ndarray, np.ndarray):
    mu = np.broadcast_to(np.asarray(mu, np.float32), (K,)).copy()
    sd = np.broadcast_to(np.asarray(sd, np.float32), (K,)).copy()
    return mu, sd


class DeepONetEngine(_Engine):
    """DeepONet VI-HMC / full-HMC log-posterior (Functional_DeepONet + GaussianNLL + Normal prior)."""
    kind = "deeponet"

    def __init__(self, spec: DeepONetSpec, branch_in, trunk_feat, y, frozen, grad_ind, prior_mu=0.0, prior_sd=0.1,
                 loss: str = "NLL", tau_out: float = 1.0, prior_scale: float = 1.0, max_chains: int = 1,
                 device="cuda"):
        super().__init__(device)
        xb = _c32(branch_in).reshape(-1, spec.in_branch)
        tf = _c32(trunk_feat).reshape(-1, spec.in_trunk)
        yy = _c32(y)
        N, P = xb.shape[0], tf.shape[0]
        if yy.shape != (N, P):
            raise ValueError(f"y must be [N={N}, P={P}] (got {yy.shape})")  # reference: assert at :144
        fz = _c32(frozen).reshape(-1)
        if fz.shape[0] != spec.n_params:
            raise ValueError(f"frozen vector must have D={spec.n_params} entries")
        idx = np.ascontiguousarray(np.asarray(grad_ind, dtype=np.int64).reshape(-1))
        K = idx.shape[0]
        pm, ps = expand_prior(K, prior_mu, prior_sd)
        self.spec, self.N, self.P = spec, N, P
        self.out_shape = (N, P)
        self.grad_ind = idx
        self._keep = (_linears(spec.branch), _linears(spec.trunk))
        d = _lib.DeepONetDesc(len(spec.branch), len(spec.trunk), self._keep[0], self._keep[1], spec.n_params, N, P,
                              spec.in_branch, spec.in_trunk, K, int(max_chains), _lik(loss, tau_out, prior_scale))
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_deeponet_plan_create(ctypes.byref(self._plan), ctypes.byref(d), _lib.fptr(xb),
                                                   _lib.fptr(tf), _lib.fptr(yy), _lib.fptr(fz), _lib.iptr(idx),
                                                   _lib.fptr(pm), _lib.fptr(ps), self.device.index)
        self._created(rc, "vihmc_deeponet_plan_create")


class MLPEngine(_Engine):
    """BNN regression log-posterior (Functional_Net + NLL/regression likelihood + Normal prior)."""
    kind = "mlp"

    def __init__(self, spec: MLPSpec, x, y, frozen, grad_ind, prior_mu=0.0, prior_sd=1.0, loss: str = "NLL",
                 tau_out: float = 0.0025, prior_scale: float = 1.0, max_chains: int = 1, device="cuda"):
        super().__init__(device)
        xx = _c32(x).reshape(-1, spec.in_dim)
        yy = _c32(y).reshape(-1, spec.out_dim)
        N = xx.shape[0]
        if yy.shape[0] != N:
            raise ValueError("x and y row counts differ")
        fz = _c32(frozen).reshape(-1)
        if fz.shape[0] != spec.n_params:
            raise ValueError(f"frozen vector must have D={spec.n_params} entries")
        idx = np.ascontiguousarray(np.asarray(grad_ind, dtype=np.int64).reshape(-1))
        K = idx.shape[0]
        pm, ps = expand_prior(K, prior_mu, prior_sd)
        self.spec, self.N = spec, N
        self.out_shape = (N, spec.out_dim)
        self.grad_ind = idx
        self._keep = _linears(spec.layers)
        d = _lib.MLPDesc(len(spec.layers), 0, self._keep, spec.n_params, N, spec.in_dim, spec.out_dim, K,
                         int(max_chains), 0, _lik(loss, tau_out, prior_scale))
        with torch.cuda.device(self.device):
            rc = self.L.vihmc_mlp_plan_create(ctypes.byref(self._plan), ctypes.byref(d), _lib.fptr(xx), _lib.fptr(yy),
                                              _lib.fptr(fz), _lib.iptr(idx), _lib.fptr(pm), _lib.fptr(ps),
                                              self.device.index)
        self._created(rc, "vihmc_mlp_plan_create")


def trunk_features(trunk_in) -> np.ndarray:
    """Trunk feature map computed with torch fp32 CPU ops exactly as the reference does
    (Operator_network/VI_HMC/my_make_func.py:33-36,63-65): [t, sin2πx, sin4πx, cos2πx, cos4πx].
    theta-independent, so it is evaluated once per plan."""
    x2 = torch.as_tensor(np.asarray(trunk_in, dtype=np.float32))
    if x2.dim() == 2:
        x2 = x2.unsqueeze(0)
    xs = x2[:, :, 1]
    x_bc = torch.stack([torch.sin(2 * np.pi * xs), torch.sin(4 * np.pi * xs), torch.cos(2 * np.pi * xs),
                        torch.cos(4 * np.pi * xs)], dim=2)
    x_bc = torch.cat([x2[:, :, 0].unsqueeze(dim=2), x_bc], dim=2)
    return x_bc[0].numpy()


def prior_per_tensor(tensor_sizes: Sequence[int], K: int, stds: Sequence[float]) -> np.ndarray:
    """Per-sampled-parameter prior std reproducing the reference's per-tensor slicing of the K-vector
    (Neural_network/VI_HMC/main_VI_HMC.py:107-112: ``w = params[i_prev:index+i_prev]`` walks the
    *sampled* vector with the full model's tensor sizes)."""
    sd = np.empty(K, np.float32)
    i = 0
    for n, s in zip(tensor_sizes, stds):
        sd[i:i + n] = s
        i += n
        if i >= K:
            break
    return sd

"""Synthetic inputs with the reference's shapes, and the reference's on-disk artefact formats.

The Burgers ``DeepOnet_data.mat`` is not shipped (Operator_network/Data/data.txt:1) and the VI
artefacts (``means_flattened_{uid}``, ``stds_flattened_{uid}``, ``gradient_indices_{uid}.npy``)
are produced by an offline VI run that is out of scope, so every DeepONet input is generated
here from a seed with numpy's PCG64 (stable bit stream), in exactly the layout
``util.get_burgers_data`` returns (Operator_network/VI_HMC/util.py:461-473):

* ``branch_in`` fp32 [N, 1, in_branch] -- smooth random fields (8 Fourier modes);
* ``trunk_in``  fp32 [1, P, 2] -- t-major (t, x) grid on [0,1]² (post_process_burgers.py:87-91);
* ``y``         fp32 [N, P] -- output of a seeded "teacher" DeepONet + N(0, noise²).

μ_VI is the teacher's flat parameter vector + N(0, mu_noise²), σ_VI a constant, and the
sensitive indices a sorted seeded subset of [0, D).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .layout import ACT_IDENTITY, ACT_RELU, ACT_SINE, ACT_TANH, DeepONetSpec, MLPSpec

TWO_PI = 2.0 * np.pi


def _rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def torch_linear_init(spec_layers, n_params: int, rng: np.random.Generator) -> np.ndarray:
    """PyTorch's default ``nn.Linear`` init (kaiming-uniform(a=√5) ≡ U(±1/√fan_in) for W and b),
    drawn from a numpy generator so it is reproducible without torch's RNG."""
    w = np.zeros(n_params, dtype=np.float64)
    for l in spec_layers:
        bound = 1.0 / np.sqrt(l.n_in)
        w[l.w_off:l.w_off + l.n_out * l.n_in] = rng.uniform(-bound, bound, l.n_out * l.n_in)
        if l.b_off >= 0:
            w[l.b_off:l.b_off + l.n_out] = rng.uniform(-bound, bound, l.n_out)
    return w


def _act(code: int, z: np.ndarray) -> np.ndarray:
    if code == ACT_TANH:
        return np.tanh(z)
    if code == ACT_RELU:
        return np.maximum(z, 0.0)
    if code == ACT_SINE:
        return np.sin(z)
    return z


def _mlp_np(layers, w: np.ndarray, x: np.ndarray) -> np.ndarray:
    h = x
    for l in layers:
        W = w[l.w_off:l.w_off + l.n_out * l.n_in].reshape(l.n_out, l.n_in)
        h = h @ W.T
        if l.b_off >= 0:
            h = h + w[l.b_off:l.b_off + l.n_out]
        h = _act(l.act, h)
    return h


def trunk_features_np(trunk_in: np.ndarray) -> np.ndarray:
    """[t, sin2πx, sin4πx, cos2πx, cos4πx] (Operator_network/VI_HMC/my_make_func.py:33-36,63-65)."""
    t, x = trunk_in[..., 0], trunk_in[..., 1]
    return np.stack([t, np.sin(TWO_PI * x), np.sin(2 * TWO_PI * x), np.cos(TWO_PI * x),
                     np.cos(2 * TWO_PI * x)], axis=-1)


@dataclass
class DeepONetProblem:
    spec: DeepONetSpec
    branch_in: np.ndarray       # fp32 [N, 1, in_branch]
    trunk_in: np.ndarray        # fp32 [1, P, 2]
    y: np.ndarray               # fp32 [N, P]
    mu: np.ndarray              # fp32 [D]   (means_flattened)
    sigma: np.ndarray           # fp32 [D]   (stds_flattened)
    grad_ind: np.ndarray        # int64 [K] sorted (gradient_indices)
    teacher: np.ndarray         # fp64 [D]

    @property
    def N(self) -> int:
        return self.y.shape[0]

    @property
    def P(self) -> int:
        return self.y.shape[1]

    @property
    def K(self) -> int:
        return self.grad_ind.shape[0]


def deeponet_problem(seed: int = 0, n: int = 1000, nt: int = 101, nx: int = 101,
                     spec: Optional[DeepONetSpec] = None, k: Optional[int] = 17240,
                     noise: float = 0.01, mu_noise: float = 0.01, sigma: float = 0.01) -> DeepONetProblem:
    """Seeded Burgers-shaped problem.  ``k=None`` selects every parameter (full HMC, K = D)."""
    spec = spec or DeepONetSpec()
    rng = _rng(seed)
    D = spec.n_params
    s = np.linspace(0.0, 1.0, spec.in_branch)
    modes = np.arange(1, 9)
    amp = rng.standard_normal((n, 8)) / modes
    ph = rng.uniform(0.0, TWO_PI, (n, 8))
    branch = np.einsum("nm,nms->ns", amp, np.sin(TWO_PI * modes[None, :, None] * s[None, None, :] + ph[:, :, None]))
    t = np.linspace(0.0, 1.0, nt)
    x = np.linspace(0.0, 1.0, nx)
    trunk = np.stack(np.meshgrid(t, x, indexing="ij"), axis=-1).reshape(nt * nx, 2)
    teacher = torch_linear_init(spec.branch + spec.trunk, D, rng)
    teacher[0] = 0.0  # DeepONet.b = Parameter(tensor(0.0)) (model.py:26)
    feats = trunk_features_np(trunk) if spec.impose_bc else trunk
    zb = _mlp_np(spec.branch, teacher, branch)
    zt = _mlp_np(spec.trunk, teacher, feats)
    y = zb @ zt.T + teacher[0] + noise * rng.standard_normal((n, nt * nx))
    mu = teacher + mu_noise * rng.standard_normal(D)
    sig = np.full(D, sigma)
    if k is None or k >= D:
        idx = np.arange(D, dtype=np.int64)
    else:
        idx = np.sort(rng.choice(D, size=k, replace=False)).astype(np.int64)
    return DeepONetProblem(spec, branch[:, None, :].astype(np.float32), trunk[None].astype(np.float32),
                           y.astype(np.float32), mu.astype(np.float32), sig.astype(np.float32), idx, teacher)


# --------------------------------------------------------------------------------------------
# BNN regression data (Neural_network/VI_HMC/main_VI_HMC.py:262-294)
# --------------------------------------------------------------------------------------------

_HERE = os.path.dirname(os.path.abspath(__file__))
BNN_DATA_FILE = os.path.join(_HERE, "..", "..", "tests", "golden", "bnn_data.npz")


def bnn_data(path: Optional[str] = None, n_tr: int = 20, n_val: int = 300, tau_out: float = 0.0025,
             seed: int = 0):
    """(x_train, y_train, x_val, y_val) fp32 column vectors.  Uses the reference's shipped tensors
    (``Neural_network/Data``, captured as data in ``tests/golden/bnn_data.npz``) when present;
    otherwise the reference's fallback generator (main_VI_HMC.py:277-287: noise std = tau_out)."""
    path = path or BNN_DATA_FILE
    if os.path.exists(path):
        z = np.load(path)
        return tuple(z[k].astype(np.float32) for k in ("x_train", "y_train", "x_val", "y_val"))
    rng = _rng(seed)
    x_val = np.linspace(-1.2, 1.2, n_val, dtype=np.float32).reshape(-1, 1)
    y_val = (4 * np.sin(4 * x_val) + 5 * np.cos(12 * x_val)).astype(np.float32)
    x_tr = np.concatenate([np.linspace(-1, -0.2, n_tr // 2), np.linspace(0.2, 1, n_tr // 2)]).astype(np.float32)
    x_tr = x_tr.reshape(-1, 1)
    y_tr = (4 * np.sin(4 * x_tr) + 5 * np.cos(12 * x_tr) + rng.standard_normal(x_tr.shape) * tau_out)
    return x_tr, y_tr.astype(np.float32), x_val, y_val


def bnn_init(spec: MLPSpec, seed: int = 0) -> np.ndarray:
    """Flat init of ``get_model`` with PyTorch's default Linear init from a seeded numpy stream."""
    return torch_linear_init(spec.layers, spec.n_params, _rng(seed)).astype(np.float32)


# --------------------------------------------------------------------------------------------
# Artefact files (formats of Operator_network/VI_HMC/main_VI_HMC_burgers.py:64-66,262,289)
# --------------------------------------------------------------------------------------------

def save_vi_artefacts(prior_file: str, uid: str, mu: np.ndarray, sigma: np.ndarray, grad_ind: np.ndarray):
    import torch
    os.makedirs(prior_file, exist_ok=True)
    torch.save(torch.from_numpy(np.asarray(mu, np.float32)), f"{prior_file}/means_flattened_{uid}")
    torch.save(torch.from_numpy(np.asarray(sigma, np.float32)), f"{prior_file}/stds_flattened_{uid}")
    np.save(f"{prior_file}/gradient_indices_{uid}.npy", np.asarray(grad_ind, np.int64))


def load_full_prior(prior_file: str):
    """The full-parameter HMC scripts' prior: ``{prior_file}/means_flattened`` and ``stds_flattened`` (no uid, no
    gradient indices: Operator_network/HMC/main_HMC_splitting.py:343-344, NUTS_DeepOnets.py:270-271), loaded with
    ``weights_only=True``."""
    import torch
    mu = torch.load(f"{prior_file}/means_flattened", weights_only=True, map_location="cpu")
    sd = torch.load(f"{prior_file}/stds_flattened", weights_only=True, map_location="cpu")
    return mu.numpy().astype(np.float32), sd.numpy().astype(np.float32)


def load_vi_artefacts(prior_file: str, uid: str):
    """Loads with non-executing loaders only (``weights_only=True``, ``allow_pickle=False``)."""
    import torch
    mu = torch.load(f"{prior_file}/means_flattened_{uid}", weights_only=True, map_location="cpu")
    sd = torch.load(f"{prior_file}/stds_flattened_{uid}", weights_only=True, map_location="cpu")
    idx = np.load(f"{prior_file}/gradient_indices_{uid}.npy", allow_pickle=False)
    return mu.numpy().astype(np.float32), sd.numpy().astype(np.float32), idx.astype(np.int64)

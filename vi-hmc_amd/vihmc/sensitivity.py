"""Sensitivity analysis of the VI parameters on the GPU: the step that writes ``gradient_indices_{uid}.npy``.

Mirrors, with the same names, arguments and return values:
* ``eval_std_dydw(valid_data, model, mean_params, std_params)`` -- Operator_network/VI/sensitivity.py:62-98
  (DeepONet: ``valid_data`` yields (x_branch [B,1,in], x_trunk [B,p,2], ...) batches as the reference's
  DataLoader over BurgersDataSet does, Operator_network/VI/utils.py:27-50) and
  Neural_network/VI/sensitivity.py:71-98 (BNN: ``valid_data = (x, y)``): sigma^2 * E[(df/dtheta)^2] for
  every parameter, as a float32 numpy array [D]. The torch.func.jacrev of the reference is replaced by
  the HIP pair-backprop kernels behind ``vihmc_sensitivity`` (vihmc_sens.hip).
* ``captured_var(imp, var_threshold)`` -- sensitivity.py:229-255 without the plot.
* ``run(...)`` -- sensitivity.py:258-288: scores -> sensitive indices -> ``sensitivity_scores_{uid}.npy``
  and ``gradient_indices_{uid}.npy`` (the files VI-HMC loads, main_VI_HMC_burgers.py:64-66).

Index form for the build's own pipeline: ``sensitivity_scores(model, branch_in, trunk_in, pts, mu, sigma)``
with ``pts`` [N, p] the trunk rows of each function (``sample_points`` restates BurgersDataSet's
``np.random.choice(P, p, replace=False)`` per item with a seeded generator).
"""
from __future__ import annotations

import os
from typing import Iterable, Optional

import numpy as np
import torch
import torch.nn as nn

from .engine import DeepONetEngine, MLPEngine, trunk_features
from . import bnn as _bnn
from . import operator as _op


def _np32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(torch.as_tensor(a).detach().cpu(), dtype=np.float32))


def _dev(device):
    return _op._device("cuda" if device is None else device)


def sample_points(N: int, P: int, p: int, seed: int = 0) -> np.ndarray:
    """[N, p] int32: per function, p distinct trunk rows (BurgersDataSet.__getitem__, utils.py:39-41)."""
    rng = np.random.default_rng(seed)
    return np.stack([rng.choice(P, p, replace=False) for _ in range(N)]).astype(np.int32)


def sensitivity_scores(model, branch_in, trunk_in, pts, mean_params, std_params=None, device=None) -> np.ndarray:
    """DeepONet scores in index form: outputs f[n][pts[n][k]]; trunk_in [P, 2] raw (t, x) rows."""
    spec = _op.spec_of(model)
    xb = _np32(branch_in).reshape(-1, spec.in_branch)
    mu = _np32(mean_params).reshape(-1)
    if mu.size != spec.n_params:
        raise ValueError(f"mean_params must have D={spec.n_params} entries")
    pts = np.ascontiguousarray(np.asarray(pts, dtype=np.int32))
    feats = trunk_features(_np32(trunk_in).reshape(-1, 2))
    eng = DeepONetEngine(spec, xb, feats, np.zeros((xb.shape[0], feats.shape[0]), np.float32), mu,
                         np.array([0], np.int64), 0.0, 1.0, "NLL", 1.0, max_chains=1, device=_dev(device))
    try:
        th = torch.tensor(mu[:1], device=eng.device)
        sd = None if std_params is None else _np32(std_params).reshape(-1)
        return eng.sensitivity(th, pts=pts, sigma=sd).cpu().numpy()
    finally:
        eng.close()


def _operator_batches(valid_data: Iterable):
    """Group the batches by size; per group: branch rows, deduplicated trunk rows and point lists."""
    groups = {}
    nb = 0
    for batch in valid_data:
        xb = _np32(batch[0])
        xt = _np32(batch[1])
        B, p = xt.shape[0], xt.shape[1]
        groups.setdefault((B, p), []).append((xb.reshape(B, -1), xt.reshape(B, p, 2)))
        nb += 1
    return groups, nb


def eval_std_dydw(valid_data, model, mean_params, std_params, device=None) -> np.ndarray:
    """sensitivity.py:62-98 (DeepONet) / Neural_network/VI/sensitivity.py:71-98 (BNN, valid_data=(x, y))."""
    if isinstance(model, nn.Sequential) or isinstance(model, _bnn.MLPSpec):
        return eval_std_dydw_bnn(valid_data, model, mean_params, std_params, device)
    groups, nb = _operator_batches(valid_data)
    if nb == 0:
        raise ValueError("valid_data is empty")
    total = None
    for (B, p), items in groups.items():
        xb = np.concatenate([b for b, _ in items], 0)
        xt = np.concatenate([t.reshape(-1, 2) for _, t in items], 0)
        uniq, inv = np.unique(xt, axis=0, return_inverse=True)   # shared grid rows -> one trunk row each
        pts = inv.reshape(-1).astype(np.int32).reshape(xb.shape[0], p)
        s = sensitivity_scores(model, xb, uniq, pts, mean_params, std_params, device).astype(np.float64)
        # the reference averages per-batch means: each size group weighs (its batches / all batches)
        s *= len(items) / nb
        total = s if total is None else total + s
    return total.astype(np.float32)


def eval_std_dydw_bnn(valid_data, model, mean_params, std_params, device=None) -> np.ndarray:
    """Neural_network/VI/sensitivity.py:71-98: x = valid_data[0], mean over all rows and outputs."""
    spec = model if isinstance(model, _bnn.MLPSpec) else _bnn.spec_of(model)
    x = _np32(valid_data[0]).reshape(-1, spec.in_dim)
    mu = _np32(mean_params).reshape(-1)
    D = spec.n_params
    eng = MLPEngine(spec, x, np.zeros((x.shape[0], spec.out_dim), np.float32), mu, np.arange(D), 0.0, 1.0, "NLL",
                    1.0, max_chains=1, device=_dev(device))
    try:
        sd = None if std_params is None else _np32(std_params).reshape(-1)
        return eng.sensitivity(torch.tensor(mu, device=eng.device), sigma=sd).cpu().numpy()
    finally:
        eng.close()


def captured_var(imp, var_threshold):
    """Number of parameters whose sorted cumulative share of sum(imp) stays <= var_threshold
    (sensitivity.py:229-255; the plot is dropped)."""
    tot_var = sum(imp)
    cumilative_sum = np.cumsum(np.sort(imp)[::-1])
    return sum(cumilative_sum / tot_var <= var_threshold)


def select_indices(imp, var_threshold) -> np.ndarray:
    """run(): ind = sort(argsort(-imp)[:num_params]) (sensitivity.py:274-281)."""
    num_params = captured_var(imp, var_threshold)
    ind = np.argsort(-imp)[:num_params]
    return np.sort(ind)


def run(valid_data, model, mean_params, std_params, save_loc: str, uid: str, importance_threshold: float = 0.90,
        device=None, load_saved_sens: bool = False) -> np.ndarray:
    """sensitivity.run without plots: writes sensitivity_scores_{uid}.npy and gradient_indices_{uid}.npy."""
    os.makedirs(save_loc, exist_ok=True)
    if load_saved_sens:
        scores = np.load(os.path.join(save_loc, f"sensitivity_scores_{uid}.npy"))
    else:
        scores = eval_std_dydw(valid_data, model, mean_params, std_params, device)
    ind = select_indices(scores, importance_threshold)
    np.save(os.path.join(save_loc, f"sensitivity_scores_{uid}.npy"), scores)
    np.save(os.path.join(save_loc, f"gradient_indices_{uid}.npy"), ind)
    return ind

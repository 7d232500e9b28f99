#!/usr/bin/env python3
"""Bayesian DeepONet VI training + sensitivity step on Burgers -- mirrors Operator_network/VI/main_VI_deeponet.py
(run :130-203) and Operator_network/VI/sensitivity.py (run :258-288) on the HIP engine:

    python vi-hmc_amd/scripts/main_VI_deeponet.py [--epochs E --n-train N]

Data: the seeded synthetic Burgers-shaped problem (the .mat is not shipped). Writes, under cfg.save_loc,
means_flattened_{uid} / stds_flattened_{uid} (best validation epoch), sensitivity_scores_{uid}.npy and
gradient_indices_{uid}.npy: the artefacts main_VI_HMC_burgers.py loads.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc import configs  # noqa: E402
from vihmc import sensitivity as S  # noqa: E402
from vihmc import vi  # noqa: E402
from vihmc.data import deeponet_problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--n-train", type=int, default=None)
    ap.add_argument("--n-valid", type=int, default=None)
    args = ap.parse_args()
    cfg = configs.load("burgers_vi")
    if args.epochs is not None:
        cfg.epochs = args.epochs
    if args.n_train is not None:
        cfg.N_train = args.n_train
    if args.n_valid is not None:
        cfg.N_valid = args.n_valid
    torch.manual_seed(cfg.seed)
    prob = deeponet_problem(seed=cfg.seed, n=cfg.N_train + cfg.N_valid)
    grid = prob.trunk_in[0]
    tr = vi.BurgersDataSet(prob.branch_in[:cfg.N_train], grid, prob.y[:cfg.N_train], cfg.p, seed=cfg.seed)
    va = vi.BurgersDataSet(prob.branch_in[cfg.N_train:], grid, prob.y[cfg.N_train:], cfg.p, seed=cfg.seed + 1)
    train_loader = torch.utils.data.DataLoader(tr, batch_size=cfg.batch_size, shuffle=True)
    valid_loader = torch.utils.data.DataLoader(va, batch_size=cfg.batch_size)
    t0 = time.perf_counter()
    model, metrics = vi.run(cfg, train_loader, valid_loader, cfg.N_train * grid.shape[0], cfg.N_valid * grid.shape[0],
                            grid)
    print(f"VI training: {cfg.epochs} epochs in {time.perf_counter() - t0:.1f} s")
    # sensitivity step on the validation functions, p random points each (config_sens.py:16-21)
    mu = torch.load(f"{cfg.save_loc}/means_flattened_{cfg.uid}", weights_only=True)
    sd = torch.load(f"{cfg.save_loc}/stds_flattened_{cfg.uid}", weights_only=True)
    pts = S.sample_points(cfg.N_valid, grid.shape[0], cfg.sens_p, seed=cfg.seed + 2)
    t0 = time.perf_counter()
    scores = S.sensitivity_scores(model.spec, prob.branch_in[cfg.N_train:], grid, pts, mu, sd)
    ind = S.select_indices(scores, cfg.importance_threshold)
    np.save(f"{cfg.save_loc}/sensitivity_scores_{cfg.uid}.npy", scores)
    np.save(f"{cfg.save_loc}/gradient_indices_{cfg.uid}.npy", ind)
    print(f"sensitivity: {time.perf_counter() - t0:.2f} s, {ind.size} sensitive parameters of {scores.size}")


if __name__ == "__main__":
    main()

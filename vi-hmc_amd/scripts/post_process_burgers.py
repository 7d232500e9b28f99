#!/usr/bin/env python3
"""Offline pooling of saved VI-HMC chains -- mirrors Operator_network/VI_HMC/post_process_burgers.py
(get_list_fnames :261-282, the pool of hmc_params_{uid}.npy[burn:] :285-288, print_error :124-146,
l2_relative_error :105-121) on the HIP engine: every pooled sample's prediction on the validation set in
batches of 16 per launch, the per-sample per-function relative L2 errors print_error reports, and the
posterior-predictive mean with its relative L2 error. Plotting / animation are out of scope.

    python vi-hmc_amd/scripts/post_process_burgers.py [--out-dir samples/Burgers/]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc import configs  # noqa: E402
from vihmc.data import load_vi_artefacts  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.operator import DeepONet, get_burgers_data  # noqa: E402
from vihmc.postprocess import get_list_fnames, load_pooled_samples, predictive, print_summary  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-dir", default=None)
    ap.add_argument("--burn", type=int, default=None)
    ap.add_argument("--n-train", type=int, default=None)
    args = ap.parse_args()
    over = {"out_dir": args.out_dir.rstrip("/") + "/"} if args.out_dir else {}
    if args.n_train:
        over.update(N_train=args.n_train, N_valid=args.n_train)
    if args.burn is not None:
        over["burn"] = args.burn
    cfg = configs.load("burgers_vi_hmc", **over)
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    uids = get_list_fnames(cfg.out_dir)
    samples = load_pooled_samples(cfg.out_dir, uids, cfg.burn)
    print(f"pooled {len(uids)} runs, {sum(s.shape[0] for s in samples)} post-burn samples")
    net = DeepONet(cfg.width_branch, cfg.width_trunk, cfg.in_branch, cfg.in_trunk, cfg.branch_depth, cfg.trunk_depth,
                   cfg.activation, cfg.output_neurons)
    mu, sigma, grad_ind = load_vi_artefacts(cfg.prior_file, cfg.prior_uid)
    _, (x1, x2, yv) = get_burgers_data(cfg)
    eng = DeepONetEngine(net.spec, x1.numpy(), trunk_features(x2), yv.numpy(), mu, grad_ind, 0.0, cfg.prior_var ** 0.5,
                         cfg.loss, cfg.tau_out, max_chains=16, device=dev)
    p = predictive(eng, samples, yv, with_rel_l2=True)
    print_summary(p, yv, with_rel_l2=True)
    np.save(f"{cfg.out_dir}posterior_mean_pooled.npy", p.mean().cpu().numpy().astype(np.float32))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Plain HMC on all 141 parameters of the BNN regression net -- mirrors Neural_network/HMC/main_regression_hmc.py
(draw_hmc_samples :102-127, validate :130-176) with Neural_network/HMC/config.py (vihmc/configs/nn_hmc.py):
hamiltorch.sample_model with model_loss='regression' (precision tau_out = 400), prior N(0, tau^-1/2) per
tensor, L = 643, step 1e-4. BASELINE config 1.

    python vi-hmc_amd/scripts/main_regression_hmc.py [--num-samples S] [--test DTSTRING]

Outputs hmc_params_{dtstring}.npy ([S_ret, 141] fp32, the reference's format) in cfg.out_dir; ``--test``
(cfg.test) validates saved samples instead: predictions on the 300 validation points from samples[burn:].
"""
import argparse
import os
import sys
from datetime import datetime

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc import bnn, configs  # noqa: E402


def draw_hmc_samples(cfg, dtstring, dev):
    torch.manual_seed(cfg.seed)
    net = bnn.get_model(cfg, cfg.bias)
    params_init = bnn.flatten(net).detach().to(dev).clone()
    print("Parameter size: ", params_init.shape[0])
    tau_list = torch.tensor([cfg.tau] * len(list(net.parameters()))).to(dev)
    x_train, y_train, _, _ = bnn.get_data(cfg)
    params_hmc = bnn.sample_model(net, x_train.to(dev), y_train.to(dev), model_loss="regression",
                                  params_init=params_init, num_samples=cfg.num_samples, step_size=cfg.step_size,
                                  num_steps_per_sample=cfg.L, tau_out=cfg.tau_out, normalizing_const=cfg.N_tr,
                                  tau_list=tau_list)
    np.save(f"{cfg.out_dir}/hmc_params_{dtstring}.npy", torch.stack(params_hmc).cpu().numpy())
    return params_hmc


def validate(cfg, dtstring, dev):
    net = bnn.get_model(cfg, cfg.bias)
    _, _, x_val, y_val = bnn.get_data(cfg)
    tau_list = torch.tensor([cfg.tau] * len(list(net.parameters()))).to(dev)
    params_hmc = torch.tensor(np.load(f"{cfg.out_dir}/hmc_params_{dtstring}.npy", allow_pickle=False))
    pred_list, log_prob_list = bnn.predict_model_hamiltorch(net, params_hmc[cfg.burn:].to(dev), x_val.to(dev),
                                                            y_val.to(dev), model_loss="regression",
                                                            tau_out=cfg.tau_out, tau_list=tau_list)
    yv = y_val.to(dev)
    print("\nExpected validation log probability: {:.2f}".format(float(torch.stack(log_prob_list).mean())))
    print("\nExpected MSE: {:.2f}".format(float(((pred_list.mean(0) - yv) ** 2).mean())))
    return pred_list, log_prob_list


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-samples", type=int, default=None)
    ap.add_argument("--L", type=int, default=None)
    ap.add_argument("--test", default=None, help="dtstring of saved samples to validate (cfg.test)")
    ap.add_argument("--out-dir", default=None)
    args = ap.parse_args()
    cfg = configs.load("nn_hmc")
    if args.num_samples:
        cfg.num_samples, cfg.burn = args.num_samples, args.num_samples // 5
    if args.L:
        cfg.L = args.L
    if args.out_dir:
        cfg.out_dir = args.out_dir
    if args.test:
        cfg.test, cfg.test_dtstring = True, args.test
    os.makedirs(cfg.out_dir, exist_ok=True)
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    dt_string = datetime.now().strftime("%d%m%y%H%M%S")
    if cfg.test:
        validate(cfg, cfg.test_dtstring, dev)
    else:
        draw_hmc_samples(cfg, dt_string, dev)
        validate(cfg, dt_string, dev)


if __name__ == "__main__":
    main()

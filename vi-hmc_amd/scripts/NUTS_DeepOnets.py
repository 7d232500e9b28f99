#!/usr/bin/env python3
"""Full-parameter DeepONet HMC with dual-averaging step-size adaptation -- mirrors
Operator_network/HMC/NUTS_DeepOnets.py (run_HMC :250-304) with Operator_network/HMC/config.py
(vihmc/configs/burgers_hmc_nuts.py): hamiltorch Sampler.HMC_NUTS = HMC whose step size adapts during burn.

    python vi-hmc_amd/scripts/NUTS_DeepOnets.py [--num-samples S --burn B --chains C]

The closure keeps the reference's prior exactly, including its per-tensor Normal(0, tau * 0.5) (a variance
used as a halved std, :128-132). Chains are batched; each adapts its own step size.
"""
import argparse
import os
import sys
import time
from datetime import datetime

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc import configs  # noqa: E402
from vihmc.data import load_full_prior  # noqa: E402
from vihmc.dist import chain_seeds  # noqa: E402
from vihmc.operator import DeepONet, define_model_log_prob_nuts, flatten, get_burgers_data  # noqa: E402
from vihmc.postprocess import post_burn_per_chain, predictive, print_summary  # noqa: E402
from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner, Sampler  # noqa: E402


def run_HMC(cfg):
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    dt_string = datetime.now().strftime("%d%m%y%H%M%S")
    os.makedirs(cfg.out_dir, exist_ok=True)
    torch.manual_seed(cfg.seed)
    net = DeepONet(cfg.width_branch, cfg.width_trunk, cfg.in_branch, cfg.in_trunk, cfg.branch_depth, cfg.trunk_depth,
                   cfg.activation, cfg.output_neurons)
    sizes = [p.nelement() for p in net.parameters()]
    shapes = [p.shape for p in net.parameters()]
    if cfg.load_prior or cfg.init_prior:
        mean_params, std_params = load_full_prior(cfg.prior_file)
    tau_list = [torch.from_numpy(mean_params), torch.from_numpy(std_params)] if cfg.load_prior else \
        [torch.tensor(cfg.prior_var)] * len(sizes)
    tr_data, vld_data = get_burgers_data(cfg)
    C = cfg.num_chains
    f = define_model_log_prob_nuts(net, cfg.loss, tr_data, sizes, shapes, tau_list, cfg.tau_out, device=dev, cfg=cfg,
                                   max_chains=C)
    params_init = (torch.from_numpy(mean_params) if cfg.init_prior else flatten(net).detach()).to(dev)
    print("Number of parameters: ", params_init.shape[0])
    runner = HMCRunner(EngineEvaluator(f._vihmc_engine), params_init[None].repeat(C, 1), cfg.num_samples, cfg.L,
                       cfg.step_size, burn=cfg.burn, sampler=Sampler.HMC_NUTS,
                       rng=ChainRNG(C, params_init.numel(), dev, seeds=chain_seeds(range(C), 1000 + cfg.seed)),
                       reuse_endpoint_grad=cfg.reuse_endpoint_grad)
    start = time.time()
    for _ in range(cfg.num_samples):
        runner.step()
    torch.cuda.synchronize()
    res = runner.result()
    print("Time taken: ", time.time() - start, " final step sizes:", res.step_size)
    fval = define_model_log_prob_nuts(net, cfg.loss, vld_data, sizes, shapes, tau_list, cfg.tau_out, predict=True,
                                      device=dev, cfg=cfg, max_chains=min(16, cfg.num_samples + 1))
    # the reference predicts on every stored sample (params_hmc[:], :294)
    p = predictive(fval._vihmc_engine, post_burn_per_chain(res.samples, res.counts, 0), vld_data[2])
    print_summary(p, vld_data[2])
    for i in range(C):
        np.save(f"{cfg.out_dir}hmc_params_{dt_string}_c{i}.npy", res.samples[i, :int(res.counts[i])].cpu().numpy())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-samples", type=int, default=None)
    ap.add_argument("--burn", type=int, default=None)
    ap.add_argument("--chains", type=int, default=None)
    ap.add_argument("--out-dir", default=None)
    ap.add_argument("--prior-file", default=None,
                    help="directory holding means_flattened / stds_flattened: sets cfg.load_prior and cfg.init_prior")
    args = ap.parse_args()
    over = {}
    if args.prior_file:
        over.update(prior_file=args.prior_file.rstrip("/"), load_prior=True, init_prior=True)
    if args.num_samples:
        over.update(num_samples=args.num_samples, burn=max(1, args.num_samples // 10))
    if args.burn:
        over["burn"] = args.burn
    if args.chains:
        over["num_chains"] = args.chains
    if args.out_dir:
        over["out_dir"] = args.out_dir.rstrip("/") + "/"
    run_HMC(configs.load("burgers_hmc_nuts", **over))


if __name__ == "__main__":
    main()

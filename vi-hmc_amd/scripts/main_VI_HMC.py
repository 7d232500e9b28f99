#!/usr/bin/env python3
"""BNN VI-HMC -- mirrors Neural_network/VI_HMC/main_VI_HMC.py (draw_hmc_samples :337-381, validate
:384-447), all cfg.num_chains chains batched in one launch (the reference runs them one after another,
:458-460), sharded over ranks when launched with torch.distributed.run. ``--full-hmc`` runs the
plain-HMC baseline of Neural_network/HMC/main_regression_hmc.py (all 141 parameters, 'regression'
likelihood, hamiltorch.sample_model semantics)."""
import argparse
import os
import sys
from datetime import datetime

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vihmc import bnn, configs  # noqa: E402
from vihmc.data import load_vi_artefacts, save_vi_artefacts  # noqa: E402
from vihmc.dist import chain_block, chain_seeds  # noqa: E402
from vihmc.postprocess import pool_ranks, post_burn_per_chain, predictive  # noqa: E402
from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains  # noqa: E402


def draw_and_validate(cfg, full_hmc=False):
    rank, ws = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    uid = [datetime.now().strftime("%d%m%y%H%M%S")]
    if ws > 1:
        dist.broadcast_object_list(uid, src=0)
    uid = uid[0]
    os.makedirs(cfg.out_dir, exist_ok=True)
    x_tr, y_tr, x_val, y_val = bnn.get_data(cfg)
    torch.manual_seed(cfg.seed)
    net = bnn.get_model(cfg, cfg.bias)
    sizes = [p.nelement() for p in net.parameters()]
    shapes = [p.shape for p in net.parameters()]
    chains = chain_block(cfg.num_chains, rank, ws)
    C = len(chains)
    if full_hmc:
        tau_list = torch.full((len(sizes),), cfg.tau)
        f = bnn.define_model_log_prob_hamiltorch(net, "regression", x_tr, y_tr, sizes, shapes, tau_list, cfg.tau_out,
                                                 device=dev, max_chains=C)
        init = bnn.flatten(net).detach()
        K_idx = np.arange(init.numel())
        fval = bnn.define_model_log_prob_hamiltorch(net, "regression", x_val, y_val, sizes, shapes, tau_list,
                                                    cfg.tau_out, predict=True, device=dev, max_chains=C)
    else:
        if not os.path.exists(f"{cfg.prior_file}/means_flattened_{cfg.prior_uid}"):
            flat = bnn.flatten(net).detach().numpy()
            rng = np.random.default_rng(cfg.seed)
            mu = (flat + 0.05 * rng.standard_normal(flat.size)).astype(np.float32)
            save_vi_artefacts(cfg.prior_file, cfg.prior_uid, mu, 0.1 * np.abs(mu) + 0.01,
                              np.sort(rng.choice(flat.size, 90, replace=False)))
        mu, sd, K_idx = load_vi_artefacts(cfg.prior_file, cfg.prior_uid)
        prior_list = [torch.from_numpy(mu[K_idx]), torch.from_numpy(sd[K_idx] if cfg.load_std else
                                                                     cfg.prior_var * np.ones(K_idx.size))] \
            if cfg.load_prior else [torch.tensor(cfg.prior_var)] * len(sizes)
        f = bnn.define_model_log_prob(net, cfg.loss, x_tr, y_tr, sizes, shapes, prior_list, cfg.tau_out, device=dev,
                                      cfg=cfg, max_chains=C)
        fval = bnn.define_model_log_prob(net, cfg.loss, x_val, y_val, sizes, shapes, prior_list, cfg.tau_out,
                                         predict=True, device=dev, cfg=cfg, max_chains=C)
        init = torch.from_numpy(mu) if cfg.init_prior else bnn.flatten(net).detach()
    th0 = init[K_idx].to(dev)
    res = run_chains(EngineEvaluator(f._vihmc_engine), th0[None].repeat(C, 1), cfg.num_samples, cfg.L,
                     cfg.step_size, rng=ChainRNG(C, th0.numel(), dev, seeds=chain_seeds(chains, 1000 + cfg.seed)),
                     reuse_endpoint_grad=getattr(cfg, "reuse_endpoint_grad", True))
    for i, c in enumerate(chains):
        np.save(f"{cfg.out_dir}hmc_params_{uid}_{c}.npy", res.samples[i, :int(res.counts[i])].cpu().numpy())
    # posterior predictive from each chain's own post-burn samples (chains that hit a LogProbError store fewer);
    # prediction sums all-reduced over ranks, the sample pool itself never moves
    p = predictive(fval._vihmc_engine, post_burn_per_chain(res.samples, res.counts, cfg.burn), y_val)
    pool_ranks(p)                                          # job-wide sums and per-sample lists
    if rank == 0:
        yv = y_val.to(dev)
        print("acceptance rate per chain:", [round(float(a), 3) for a in res.accepted.float().mean(1)])
        print("\nExpected validation log probability: {:.2f}".format(float(np.mean(p.log_prob))))
        print("\nExpected MSE: {:.2f}".format(float(((p.mean().float() - yv) ** 2).mean())))
        print("\nFinal MSE: {:.2f}".format(p.mse[-1]))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full-hmc", action="store_true")
    ap.add_argument("--num-samples", type=int, default=None)
    ap.add_argument("--chains", type=int, default=None)
    args = ap.parse_args()
    cfg = configs.load("nn_hmc" if args.full_hmc else "nn_vi_hmc")
    if not args.full_hmc:
        cfg.prior_file = os.path.join(cfg.out_dir, "artefacts")
    if args.num_samples:
        cfg.num_samples, cfg.burn = args.num_samples, args.num_samples // 5
    if args.chains:
        cfg.num_chains = args.chains
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
        dist.init_process_group("nccl")
    draw_and_validate(cfg, args.full_hmc)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Full-parameter DeepONet HMC with a split Hamiltonian over data shards -- mirrors
Operator_network/HMC/main_HMC_splitting.py (get_split_data :28-76, run_HMC :323-383, validate_HMC) with
config_splitting.py (vihmc/configs/burgers_hmc_splitting.py). BASELINE config 4: one chain per GPU.

    python vi-hmc_amd/scripts/main_HMC_splitting.py [--num-samples S --chains C --n-train N]

Each of the cfg.num_splits contiguous shards (N_train / num_splits functions x all P points) gets its own
full-parameter closure with the prior divided by num_splits (define_split_model_log_prob), and
Integrator.SPLITTING runs Neal's split integrator over them (Sampler.HMC_NUTS when cfg.is_nuts). All
chains of a rank are batched in one launch per shard evaluation. Data: ../Data/DeepOnet_data.mat when
present, else the seeded synthetic Burgers-shaped problem. Outputs: hmc_params_{uid}_c{chain}.npy.
"""
import argparse
import os
import sys
import time
from datetime import datetime

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vihmc import configs  # noqa: E402
from vihmc.data import load_full_prior  # noqa: E402
from vihmc.dist import chain_block, chain_seeds  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.operator import DeepONet, define_split_model_log_prob, flatten, get_burgers_data  # noqa: E402
from vihmc.postprocess import append_fname, pool_ranks, post_burn_per_chain, predictive, print_summary  # noqa: E402
from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner, Integrator, Sampler  # noqa: E402


def get_split_data(cfg):
    """main_HMC_splitting.py:28-54: num_splits equal contiguous shards of the training functions."""
    tr, vld = get_burgers_data(cfg)
    x1, x2, y = tr
    if x1.shape[0] % cfg.num_splits != 0:
        raise ValueError("Number of splits does not split the data equally")
    n = x1.shape[0] // cfg.num_splits
    return [(x1[i * n:(i + 1) * n], x2, y[i * n:(i + 1) * n]) for i in range(cfg.num_splits)], vld


def run_HMC(cfg):
    rank, ws = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    uid = [datetime.now().strftime("%d%m%y%H%M%S")]
    if ws > 1:
        dist.broadcast_object_list(uid, src=0)
    uid = uid[0]
    os.makedirs(cfg.out_dir, exist_ok=True)
    torch.manual_seed(cfg.seed)
    net = DeepONet(cfg.width_branch, cfg.width_trunk, cfg.in_branch, cfg.in_trunk, cfg.branch_depth, cfg.trunk_depth,
                   cfg.activation, cfg.output_neurons)
    if cfg.load_prior or cfg.init_prior:
        mean_params, std_params = load_full_prior(cfg.prior_file)
    tau_list = [torch.from_numpy(mean_params), torch.from_numpy(std_params)] if cfg.load_prior else \
        [torch.tensor(cfg.prior_var)]
    tr_data, vld_data = get_split_data(cfg)
    chains = chain_block(cfg.num_chains, rank, ws)
    C = len(chains)
    # one engine per shard, each batching this rank's C chains in every launch
    fns = define_split_model_log_prob(net, cfg.loss, tr_data, cfg.num_splits, tau_list, cfg.tau_out, device=dev,
                                      verbose=rank == 0, cfg=cfg, max_chains=C)
    params_init = (torch.from_numpy(mean_params) if cfg.init_prior else flatten(net).detach()).to(dev)
    if rank == 0:
        print("Number of parameters: ", params_init.shape[0], " chains:", cfg.num_chains, " ranks:", ws)
    runner = HMCRunner([EngineEvaluator(f._vihmc_engine) for f in fns], params_init[None].repeat(C, 1),
                       cfg.num_samples, cfg.L, cfg.step_size, burn=cfg.burn if cfg.is_nuts else 0,
                       sampler=Sampler.HMC_NUTS if cfg.is_nuts else Sampler.HMC, integrator=Integrator.SPLITTING,
                       rng=ChainRNG(C, params_init.numel(), dev, seeds=chain_seeds(chains, 1000 + cfg.seed)),
                       reuse_endpoint_grad=cfg.reuse_endpoint_grad)
    start = time.time()
    for _ in range(cfg.num_samples):
        runner.step()
    torch.cuda.synchronize()
    res = runner.result()
    print(f"[rank {rank}] Time taken: {time.time() - start:.2f} s, acceptance {float(res.accepted.float().mean()):.3f}")
    for i, c in enumerate(chains):
        np.save(f"{cfg.out_dir}hmc_params_{uid}_c{c}.npy", res.samples[i, :int(res.counts[i])].cpu().numpy())
    if ws > 1:
        dist.barrier()
    if rank == 0:
        for c in range(cfg.num_chains):
            append_fname(cfg.out_dir, f"{uid}_c{c}")
    # the reference predicts on ALL samples here (no burn, main_HMC_splitting.py:373 -- App. B quirk kept)
    x1, x2, yv = vld_data
    D = net.spec.n_params
    pm, ps = (mean_params, std_params) if cfg.load_prior else (0.0, cfg.prior_var ** 0.5)
    veng = DeepONetEngine(net.spec, x1.numpy(), trunk_features(x2), yv.numpy(), np.zeros(D, np.float32),
                          np.arange(D), pm, ps, cfg.loss, cfg.tau_out, max_chains=min(16, cfg.num_samples + 1),
                          device=dev)
    p = predictive(veng, post_burn_per_chain(res.samples, res.counts, 0), yv)
    pool_ranks(p)                                          # job-wide sums and per-sample lists
    if rank == 0:
        print_summary(p, yv)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-samples", type=int, default=None)
    ap.add_argument("--chains", type=int, default=None)
    ap.add_argument("--n-train", type=int, default=None)
    ap.add_argument("--out-dir", default=None)
    ap.add_argument("--prior-file", default=None,
                    help="directory holding means_flattened / stds_flattened: sets cfg.load_prior and cfg.init_prior")
    args = ap.parse_args()
    over = {}
    if args.prior_file:
        over.update(prior_file=args.prior_file.rstrip("/"), load_prior=True, init_prior=True)
    if args.num_samples:
        over.update(num_samples=args.num_samples, burn=args.num_samples // 2)
    if args.chains:
        over["num_chains"] = args.chains
    if args.n_train:
        over.update(N_train=args.n_train, N_valid=args.n_train)
    if args.out_dir:
        over["out_dir"] = args.out_dir.rstrip("/") + "/"
    cfg = configs.load("burgers_hmc_splitting", **over)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
        dist.init_process_group("nccl")
    run_HMC(cfg)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""DeepONet VI-HMC on Burgers -- mirrors Operator_network/VI_HMC/main_VI_HMC_burgers.py
(run_VI_HMC :244-301, eval_VI_HMC :304-349) on the HIP engine, with C chains per GPU and
torch.distributed chain sharding:

    python vi-hmc_amd/scripts/main_VI_HMC_burgers.py [--num-samples S --chains C]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        vi-hmc_amd/scripts/main_VI_HMC_burgers.py --chains 128

Data: ../Data/DeepOnet_data.mat when present, else the seeded synthetic Burgers-shaped problem;
VI artefacts from cfg.prior_file/prior_uid when present, else synthetic ones are written there.
Outputs (cfg.out_dir): hmc_params_{uid}_c{chain}.npy ([S_ret, K] fp32, the reference's format),
sample_mse_{uid}.npy, and the pooled posterior-predictive mean.
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
from vihmc.data import deeponet_problem, load_vi_artefacts, save_vi_artefacts  # noqa: E402
from vihmc.dist import all_reduce_sum, chain_block, chain_seeds, gather_pool  # noqa: E402
from vihmc.operator import DeepONet, define_model_log_prob, flatten, get_burgers_data, l2_relative_error  # noqa: E402
from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner, Sampler  # noqa: E402


def artefacts(cfg, net):
    f = f"{cfg.prior_file}/means_flattened_{cfg.prior_uid}"
    if not os.path.exists(f):
        p = deeponet_problem(seed=cfg.seed, n=2, nt=2, nx=2, spec=net.spec, k=cfg.sensitive_k)
        save_vi_artefacts(cfg.prior_file, cfg.prior_uid, p.mu, p.sigma, p.grad_ind)
    return load_vi_artefacts(cfg.prior_file, cfg.prior_uid)


def run_VI_HMC(cfg):
    rank, ws = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    dt_string = datetime.now().strftime("%d%m%y%H%M%S") + "_" + str(os.environ.get("SLURM_JOB_ID"))
    os.makedirs(cfg.out_dir, exist_ok=True)
    torch.manual_seed(cfg.seed)
    net = DeepONet(cfg.width_branch, cfg.width_trunk, cfg.in_branch, cfg.in_trunk, cfg.branch_depth, cfg.trunk_depth,
                   cfg.activation, cfg.output_neurons)
    mu, sigma, grad_ind = artefacts(cfg, net)
    tau_list = [torch.from_numpy(mu[grad_ind]), torch.from_numpy(sigma[grad_ind])] if cfg.load_prior else \
        [torch.tensor(cfg.prior_var)]
    tr_data, vld_data = get_burgers_data(cfg)
    chains = chain_block(cfg.num_chains, rank, ws)
    C = len(chains)
    log_prob_func = define_model_log_prob(net, cfg.loss, tr_data, tau_list, cfg.tau_out, device=dev, cfg=cfg,
                                          max_chains=C)
    if cfg.init_prior:
        g = torch.Generator().manual_seed(cfg.seed)
        init = torch.normal(torch.from_numpy(mu), torch.from_numpy(sigma), generator=g) if cfg.sample_prior \
            else torch.from_numpy(mu)
    else:
        init = flatten(net).detach()
    params_init = init[grad_ind].to(dev)
    if rank == 0:
        print("Number of parameters: ", params_init.shape[0], " chains:", cfg.num_chains, " ranks:", ws)
    runner = HMCRunner(EngineEvaluator(log_prob_func._vihmc_engine), params_init[None].repeat(C, 1), cfg.num_samples,
                       cfg.L, cfg.step_size, sampler=Sampler.HMC,
                       rng=ChainRNG(C, params_init.numel(), dev, seeds=chain_seeds(chains, 1000 + cfg.seed)),
                       reuse_endpoint_grad=cfg.reuse_endpoint_grad)
    start = time.time()
    for _ in range(cfg.num_samples):
        runner.step()
    torch.cuda.synchronize()
    took = time.time() - start
    res = runner.result()
    print(f"[rank {rank}] Time taken: {took:.2f} s, acceptance {float(res.accepted.float().mean()):.3f}")
    for i, c in enumerate(chains):
        np.save(f"{cfg.out_dir}hmc_params_{dt_string}_c{c}.npy", res.samples[i, :int(res.counts[i])].cpu().numpy())
    pool = gather_pool(res.stacked())                      # one RCCL all-gather over xGMI
    # posterior predictive on the validation set, this rank's chains, summed over ranks
    from vihmc.engine import DeepONetEngine, trunk_features
    x1, x2, yv = vld_data
    veng = DeepONetEngine(net.spec, x1.numpy(), trunk_features(x2), yv.numpy(), mu, grad_ind,
                          *((mu[grad_ind], sigma[grad_ind]) if cfg.load_prior else (0.0, cfg.prior_var ** 0.5)),
                          loss=cfg.loss, tau_out=cfg.tau_out, max_chains=min(16, C * cfg.num_samples), device=dev)
    local = res.stacked()[:, cfg.burn:].reshape(-1, params_init.numel())
    psum = torch.zeros(yv.shape, dtype=torch.float64, device=dev)
    mse, lps = [], []
    y_dev = yv.to(dev)
    with torch.no_grad():
        for s in range(0, local.shape[0], veng.max_chains):
            lp, out = veng.forward(local[s:s + veng.max_chains])
            psum += out.double().sum(0)
            mse += ((out - y_dev) ** 2).mean((1, 2)).tolist()
            lps += lp.tolist()
    n = torch.tensor([float(local.shape[0])], dtype=torch.float64, device=dev)
    all_reduce_sum(psum)
    all_reduce_sum(n)
    if rank == 0:
        mean = (psum / n).cpu().numpy()
        err = l2_relative_error(yv.numpy().astype(np.float64), mean)
        print("\nExpected validation log probability: {:.2f}".format(np.mean(lps)))
        print("\nExpected MSE: {:.4f}".format(np.mean(mse)))
        print("\nFinal MSE: {:.4f}".format(mse[-1]))
        print("\nMin MSE:{:.6f}".format(min(mse)))
        print("\nMean relative L2 error of the posterior-predictive mean: {:.5f}".format(err.mean()))
        np.save(f"{cfg.out_dir}sample_mse_{dt_string}.npy", np.asarray(mse))
        np.save(f"{cfg.out_dir}posterior_mean_{dt_string}.npy", mean.astype(np.float32))
        print("pooled samples:", tuple(pool.shape))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-samples", type=int, default=None)
    ap.add_argument("--chains", type=int, default=None)
    ap.add_argument("--n-train", type=int, default=None)
    args = ap.parse_args()
    over = {}
    if args.num_samples:
        over.update(num_samples=args.num_samples, burn=min(args.num_samples // 10, 100))
    if args.chains:
        over["num_chains"] = args.chains
    if args.n_train:
        over.update(N_train=args.n_train, N_valid=args.n_train)
    cfg = configs.load("burgers_vi_hmc", **over)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
        dist.init_process_group("nccl")
    run_VI_HMC(cfg)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

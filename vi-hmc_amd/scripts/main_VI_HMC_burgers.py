#!/usr/bin/env python3
"""DeepONet VI-HMC on Burgers -- mirrors Operator_network/VI_HMC/main_VI_HMC_burgers.py
(run_VI_HMC :244-301, eval_VI_HMC :304-349) on the HIP engine, with C chains per GPU and
torch.distributed chain sharding:

    python vi-hmc_amd/scripts/main_VI_HMC_burgers.py [--num-samples S --chains C]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        vi-hmc_amd/scripts/main_VI_HMC_burgers.py --chains 128

Data: ../Data/DeepOnet_data.mat when present, else the seeded synthetic Burgers-shaped problem;
VI artefacts from cfg.prior_file/prior_uid when present, else synthetic ones are written there.
Outputs (cfg.out_dir): hmc_params_{uid}_c{chain}.npy ([S_ret, K] fp32, the reference's format), one line
"{uid}_c{chain}" per chain appended to fnames.txt (what post_process_burgers.py pools), sample_mse_{uid}.npy,
and the posterior-predictive mean. ``--evaluate UID`` (cfg.evaluate / cfg.eval_dt_string) re-evaluates saved
samples instead of sampling (eval_VI_HMC, :304-349); ``--gather-pool`` also all-gathers the whole sample pool
to every rank (RCCL over xGMI; off by default: only prediction sums are reduced).
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
from vihmc.dist import chain_block, chain_seeds, gather_ragged_pool  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.operator import DeepONet, define_model_log_prob, flatten, get_burgers_data  # noqa: E402
from vihmc.postprocess import (append_fname, load_pooled_samples, pool_ranks, post_burn_per_chain,  # noqa: E402
                               predictive, print_summary)
from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner, Sampler  # noqa: E402


def artefacts(cfg, net):
    f = f"{cfg.prior_file}/means_flattened_{cfg.prior_uid}"
    if not os.path.exists(f):
        p = deeponet_problem(seed=cfg.seed, n=2, nt=2, nx=2, spec=net.spec, k=cfg.sensitive_k)
        save_vi_artefacts(cfg.prior_file, cfg.prior_uid, p.mu, p.sigma, p.grad_ind)
    return load_vi_artefacts(cfg.prior_file, cfg.prior_uid)


def run_VI_HMC(cfg, gather=False):
    rank, ws = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    dt_string = [datetime.now().strftime("%d%m%y%H%M%S") + "_" + str(os.environ.get("SLURM_JOB_ID"))]
    if ws > 1:
        dist.broadcast_object_list(dt_string, src=0)       # one uid for the whole job's files
    dt_string = dt_string[0]
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
    if ws > 1:
        dist.barrier()
    if rank == 0:
        for c in range(cfg.num_chains):
            append_fname(cfg.out_dir, f"{dt_string}_c{c}")
    if gather:
        # one RCCL all-gather over xGMI; chains store different counts after a LogProbError
        pool, pool_counts = gather_ragged_pool(res.samples, res.counts)
        if rank == 0:
            print("pooled samples:", tuple(pool.shape), "stored per chain:", pool_counts.tolist())
    # posterior predictive on the validation set: this rank's chains (each its own post-burn samples),
    # prediction sums all-reduced over ranks
    evaluate(cfg, net.spec, mu, sigma, grad_ind, vld_data, post_burn_per_chain(res.samples, res.counts, cfg.burn),
             dev, rank, tag=dt_string)
    return res


def evaluate(cfg, spec, mu, sigma, grad_ind, vld_data, sample_sets, dev, rank, tag):
    x1, x2, yv = vld_data
    n_max = max(1, max((s.shape[0] for s in sample_sets), default=1))
    veng = DeepONetEngine(spec, x1.numpy(), trunk_features(x2), yv.numpy(), mu, grad_ind,
                          *((mu[grad_ind], sigma[grad_ind]) if cfg.load_prior else (0.0, cfg.prior_var ** 0.5)),
                          loss=cfg.loss, tau_out=cfg.tau_out, max_chains=min(16, n_max), device=dev)
    p = predictive(veng, sample_sets, yv)
    pool_ranks(p)                                          # job-wide sums and per-sample lists
    if rank == 0 and p.mse:
        print_summary(p, yv)
        np.save(f"{cfg.out_dir}sample_mse_{tag}.npy", np.asarray(p.mse))
        np.save(f"{cfg.out_dir}posterior_mean_{tag}.npy", p.mean().cpu().numpy().astype(np.float32))
    veng.close()
    return p


def eval_VI_HMC(cfg, dt_string):
    """main_VI_HMC_burgers.py:304-349: predictive of the saved hmc_params_{dt_string}.npy[burn:] (a uid of
    fnames.txt, e.g. '<dt>_c0')."""
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    net = DeepONet(cfg.width_branch, cfg.width_trunk, cfg.in_branch, cfg.in_trunk, cfg.branch_depth, cfg.trunk_depth,
                   cfg.activation, cfg.output_neurons)
    mu, sigma, grad_ind = load_vi_artefacts(cfg.prior_file, cfg.prior_uid)
    _, vld_data = get_burgers_data(cfg)
    sets = load_pooled_samples(cfg.out_dir.rstrip("/"), [dt_string], cfg.burn)
    return evaluate(cfg, net.spec, mu, sigma, grad_ind, vld_data, sets, dev, 0, tag=f"eval_{dt_string}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-samples", type=int, default=None)
    ap.add_argument("--chains", type=int, default=None)
    ap.add_argument("--n-train", type=int, default=None)
    ap.add_argument("--evaluate", default=None, help="uid of saved samples to evaluate (cfg.evaluate)")
    ap.add_argument("--gather-pool", action="store_true")
    ap.add_argument("--out-dir", default=None)
    ap.add_argument("--burn", type=int, default=None)
    args = ap.parse_args()
    over = {}
    if args.num_samples:
        over.update(num_samples=args.num_samples, burn=min(args.num_samples // 10, 100))
    if args.chains:
        over["num_chains"] = args.chains
    if args.n_train:
        over.update(N_train=args.n_train, N_valid=args.n_train)
    if args.burn is not None:
        over["burn"] = args.burn
    if args.evaluate:
        over.update(evaluate=True, eval_dt_string=args.evaluate)
    if args.out_dir:
        over["out_dir"] = args.out_dir.rstrip("/") + "/"
    cfg = configs.load("burgers_vi_hmc", **over)
    if cfg.evaluate:
        print("Evaluating...")
        eval_VI_HMC(cfg, cfg.eval_dt_string)
        return
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
        dist.init_process_group("nccl")
    run_VI_HMC(cfg, gather=args.gather_pool)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

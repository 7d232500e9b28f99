"""Child of tests/test_gpu_dist.py, launched as `python -m torch.distributed.run --nproc-per-node 1 ...` (the
driver's multi-GPU launch form): one rank on cuda:LOCAL_RANK with the ``nccl`` backend (RCCL), the batched HIP
sampler on its chain block (vihmc.dist.chain_block / chain_seeds), then the pool all-gather and the accept-count
all-reduce issued as real RCCL collectives (vihmc.dist short-circuits them at world size 1, so they are called
through torch.distributed directly here). Saves the gathered pool for the parent to compare."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (HERE, os.path.join(HERE, ".."), os.path.join(HERE, "..", "vi-hmc_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--chains", type=int, default=2)
    args = ap.parse_args()
    local = int(os.environ["LOCAL_RANK"])
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from goldens import deeponet_case
    from vihmc.dist import chain_block, chain_seeds
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    c = deeponet_case("deeponet_small")
    p = c.prob
    chains = chain_block(args.chains, rank, ws)
    C = len(chains)
    eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                         c.prior_sd, c.loss, c.tau_out, max_chains=C, device=dev)
    th0 = torch.tensor(np.asarray(c.thetas[0]))
    res = run_chains(EngineEvaluator(eng), th0[None].repeat(C, 1), 6, 7, 2e-3,
                     rng=ChainRNG(C, th0.numel(), dev, seeds=chain_seeds(chains)))
    local_pool = res.stacked().to(dev).contiguous()
    pool = torch.empty((ws * C,) + tuple(local_pool.shape[1:]), device=dev, dtype=local_pool.dtype)
    dist.all_gather_into_tensor(pool, local_pool)
    acc = res.accepted.to(dev).sum().reshape(1).to(torch.float64)
    dist.all_reduce(acc, op=dist.ReduceOp.SUM)
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"pool": pool.cpu(), "acc": acc.cpu(), "backend": dist.get_backend()}, args.out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

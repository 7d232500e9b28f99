"""world_size-2 gloo test of the chain-parallel path on the CPU: every rank samples its chain block
with per-chain seeds and the all-gathered pool equals the single-process run of all chains."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vihmc.dist import chain_block, chain_seeds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sample(chains, tmp_unused=None):
    from test_sampler import bnn_fn
    from vihmc import samplers as S
    fn, th0, _ = bnn_fn()
    C = len(chains)
    res = S.run_chains(S.AutogradEvaluator(fn, th0.numel(), "cpu"), th0[None].repeat(C, 1), 6, 4, 5e-4, burn=1,
                       rng=S.ChainRNG(C, th0.numel(), "cpu", seeds=chain_seeds(chains)))
    return res


def _worker(rank, ws, port, total, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(here, ".."), os.path.join(here, "..", "vi-hmc_amd")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from vihmc.dist import all_reduce_sum, gather_pool
    chains = chain_block(total, rank, ws)
    res = _sample(chains)
    pool = gather_pool(res.stacked())
    acc = all_reduce_sum(res.accepted.sum().reshape(1).to(torch.float64))
    if rank == 0:
        torch.save({"pool": pool, "acc": acc}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_chain_block_partition():
    for total in (1, 5, 16, 128):
        for ws in (1, 2, 3, 8):
            blocks = [chain_block(total, r, ws) for r in range(ws)]
            ids = [c for b in blocks for c in b]
            assert ids == list(range(total))


@pytest.mark.parametrize("total", [4, 5])
def test_gloo_world2_pool_equals_single_process(tmp_path, total):
    out = str(tmp_path / "pool.pt")
    mp.start_processes(_worker, args=(2, _free_port(), total, out), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    ref = _sample(range(total))
    assert torch.equal(got["pool"], ref.stacked())
    assert float(got["acc"][0]) == float(ref.accepted.sum())

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


class _NaNAt:
    """Wraps a CPU evaluator: chain 0's log-prob is NaN on gradient call number ``at`` (a LogProbError: the
    sampler rejects without storing, so that chain ends with fewer stored samples than the others)."""

    def __init__(self, ev, at):
        self.ev, self.at, self.calls = ev, at, 0
        self.device, self.K = ev.device, ev.K

    def logp_grad(self, theta):
        lp, g = self.ev.logp_grad(theta)
        self.calls += 1
        if self.calls == self.at:
            lp = lp.clone()
            lp[0] = float("nan")
        return lp, g

    def logp(self, theta):
        return self.ev.logp(theta)


def _bench_worker(rank, ws, port, out_path):
    """bench.py's multi-rank tail on gloo: per-rank runner, ragged pool all-gather, max-over-ranks wall."""
    import sys
    import time
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(here, ".."), os.path.join(here, "..", "vi-hmc_amd")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from test_sampler import bnn_fn
    from vihmc import samplers as S
    from vihmc.dist import gather_ragged_pool, max_over_ranks
    fn, th0, _ = bnn_fn()
    chains = chain_block(5, rank, ws)
    C = len(chains)
    ev = S.AutogradEvaluator(fn, th0.numel(), "cpu")
    if rank == 1:
        ev = _NaNAt(ev, at=9)                          # rank 1, its first chain: one LogProbError mid-run
    runner = S.HMCRunner(ev, th0[None].repeat(C, 1), 8, 4, 5e-4, burn=0,
                         rng=S.ChainRNG(C, th0.numel(), "cpu", seeds=chain_seeds(chains)), strict_rng=True)
    t0 = time.perf_counter()
    for _ in range(8):
        runner.step()
    wall = time.perf_counter() - t0 + (0.25 if rank == 1 else 0.0)
    T = max_over_ranks(wall, "cpu")
    pool, counts = gather_ragged_pool(runner.samples, runner.counts)
    local = [runner.samples[i, :int(runner.counts[i])].clone() for i in range(C)]
    torch.save({"pool": pool, "counts": counts, "local": local, "T": T, "wall": wall},
               out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_bench_pool_with_logprob_error(tmp_path):
    out = str(tmp_path / "bench")
    mp.start_processes(_bench_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    # the job's time is the slowest rank's, on every rank
    assert r0["T"] == r1["T"] == max(r0["wall"], r1["wall"])
    # ragged: rank 1's first chain (job chain 3) stored one sample fewer than the rest
    counts = r0["counts"].tolist()
    assert counts == r1["counts"].tolist() and len(counts) == 5
    assert counts[3] == counts[0] - 1 and len({counts[i] for i in (0, 1, 2, 4)}) == 1
    assert torch.equal(r0["pool"], r1["pool"])
    local = r0["local"] + r1["local"]
    for c in range(5):
        n = counts[c]
        assert torch.equal(r0["pool"][c, :n], local[c])
        assert not r0["pool"][c, n:].any()                # padding
